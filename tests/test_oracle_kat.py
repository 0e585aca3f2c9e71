"""Pins the CPU oracle (C) and the independent Python restatement against every
known-answer vector in the reference's own unit tests (tests/golden/reference_kats.json).
"""
import pytest

from oracle import coracle, pyoracle
from tests import kats

IMPLS = {"c": coracle, "py": pyoracle}


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("v", kats.by_kind("sum_be_words"), ids=lambda v: v["name"])
def test_sum_be_words(impl, v):
    assert IMPLS[impl].sum_be_words(v["data"], v["skipword"]) == v["expected"]


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("v", kats.by_kind("checksum"), ids=lambda v: v["name"])
def test_checksum(impl, v):
    assert IMPLS[impl].checksum(v["data"], v["skipword"]) == v["expected"]


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("v", kats.by_kind("ipv4_checksum", "ipv6_checksum"), ids=lambda v: v["name"])
def test_pseudo_header_checksum(impl, v):
    fn = IMPLS[impl].ipv4_checksum if v["kind"] == "ipv4_checksum" else IMPLS[impl].ipv6_checksum
    got = fn(v["data"], v["skipword"], b"", bytes(v["src"]), bytes(v["dst"]), v["proto"])
    assert got == v["expected"]


def _frame(ip_payload, ethertype):
    return bytes(12) + ethertype.to_bytes(2, "big") + bytes(ip_payload)


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("v", kats.by_kind("ipv4_header"), ids=lambda v: v["name"])
def test_ipv4_header_checksum_via_rx(impl, v):
    # ipv4::checksum(&Ipv4Packet) is what the receive path computes on eth.payload()
    r = IMPLS[impl].rx_frame(_frame(v["data"], 0x0800))
    assert r["ip_csum"] == v["expected"]


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("v", kats.by_kind("ipv4_payload_len"), ids=lambda v: v["name"])
def test_ipv4_payload_len(impl, v):
    d = bytearray(v["data"])
    d[9] = 253  # Test1 protocol: dispatch stops after the payload bounds
    r = IMPLS[impl].rx_frame(_frame(d, 0x0800))
    assert r["l4_length"] == v["expected"]


@pytest.mark.parametrize("impl", sorted(IMPLS))
def test_ipv6_payload_len(impl):
    (v,) = kats.by_kind("ipv6_payload_len")
    r = IMPLS[impl].rx_frame(_frame(v["data"], 0x86DD))
    assert r["l4_length"] == v["expected"] and r["l4_offset"] == 54


@pytest.mark.parametrize("impl", sorted(IMPLS))
def test_ethernet_fields(impl):
    (v,) = kats.by_kind("ethernet_fields")
    r = IMPLS[impl].rx_frame(v["data"])
    assert r["ethertype"] == v["expected"]["ethertype"]
    # Ethernet-only frame (payload empty) carrying the IPv6 ethertype: Ipv6Packet::new fails
    assert r["status"] & pyoracle.ST_L3_MALFORMED


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("v", kats.by_kind("rx_frame"), ids=lambda v: v["name"])
def test_rx_frame_derived(impl, v):
    r = IMPLS[impl].rx_frame(v["data"])
    e = v["expected"]
    for k in ("ip_csum", "l4_csum", "l4_offset", "l4_length", "src_port", "dst_port"):
        assert r[k] == e[k], k
    assert bool(r["status"] & pyoracle.ST_IP_CSUM_OK) == e["ip_ok"]
    assert bool(r["status"] & pyoracle.ST_L4_CSUM_OK) == e["l4_ok"]


def test_rec_layout():
    assert coracle.lib().oracle_rec_size() == coracle.REC_DTYPE.itemsize


@pytest.mark.parametrize("impl", sorted(IMPLS))
@pytest.mark.parametrize("v", kats.by_kind("getters"), ids=lambda v: v["name"])
def test_header_getters(impl, v):
    """Every generated getter the record carries equals the value the reference's
    test asserts (ethernet.rs, ipv4.rs, ipv6.rs, udp.rs, tcp.rs), and the fields
    of views the dispatch did not reach stay 0."""
    r = IMPLS[impl].rx_frame(kats.getter_frame(v))
    for k, want in v["expected"].items():
        assert int(r[k]) == want, k
    if v["view"] != "tcp":
        assert int(r["tcp_sequence"]) == 0 and int(r["tcp_window"]) == 0
    if v["view"] not in ("ipv6", "icmpv6"):
        assert int(r["ip6_flow_label"]) == 0 and int(r["ip6_traffic_class"]) == 0
