"""The reference's own unit tests, restated against libpnet_amd.packet (the
pnet_packet function names, computed on the GPU). Each test cites the
reference test it mirrors; expected values come from those tests (via
tests/golden/reference_kats.json where the survey captured them)."""
import ipaddress

import numpy as np
import pytest

from libpnet_amd.packet import icmp, icmpv6, ipv4, tcp, udp, util
from oracle import coracle
from tests import kats

pytestmark = pytest.mark.gpu


def test_util_checksum_kats():
    # util.rs:189-237 (sum_be_words via checksum) and icmp.rs:82-108
    for v in kats.by_kind("checksum"):
        assert util.checksum(v["data"], v["skipword"]) == v["expected"], v["name"]
    for v in kats.by_kind("sum_be_words"):
        want = 0 if not v["data"] else (~_fold(v["expected"])) & 0xFFFF
        assert util.checksum(v["data"], v["skipword"]) == want, v["name"]


def _fold(s):
    while s >> 16:
        s = (s >> 16) + (s & 0xFFFF)
    return s


def test_ipv4_checksum_header_tests():
    # ipv4.rs:185-223 (zeros, nonzero, too small / too large IHL) and 292-357
    for v in kats.by_kind("ipv4_header"):
        assert ipv4.checksum(v["data"]) == v["expected"], v["name"]


def test_udp_checksums():
    # udp.rs:58-100 (IPv4) and 128-170 (IPv6)
    v4 = next(v for v in kats.by_kind("ipv4_checksum") if v["name"] == "udp_ipv4_checksum")
    assert udp.ipv4_checksum(v4["data"], ipaddress.IPv4Address("192.168.0.1"),
                             ipaddress.IPv4Address("192.168.0.199")) == v4["expected"] == 0x9178
    v6 = next(v for v in kats.by_kind("ipv6_checksum") if v["name"] == "udp_ipv6_checksum")
    assert udp.ipv6_checksum(v6["data"], "::1", "::1") == v6["expected"]


def test_tcp_ipv4_checksum():
    # tcp.rs:288-357
    v = next(v for v in kats.by_kind("ipv4_checksum") if v["name"] == "tcp_ipv4_checksum")
    assert tcp.ipv4_checksum(v["data"], "192.168.2.1", "192.168.111.51") == v["expected"]


def test_icmp_and_icmpv6():
    # icmp.rs:82-108, icmpv6.rs:88-117
    for v in kats.by_kind("checksum"):
        if v["name"].startswith("icmp"):
            assert icmp.checksum(v["data"]) == v["expected"], v["name"]
    for v in kats.by_kind("ipv6_checksum"):
        if v["name"].startswith("icmpv6"):
            assert icmpv6.checksum(v["data"], bytes(v["src"]), bytes(v["dst"])) == v["expected"], v["name"]


def test_adv_forms_and_batches_match_oracle():
    # udp.rs:45-56 / tcp.rs:250-261 (extra_data), checked against the restatement
    rng = np.random.default_rng(9)
    datas = [rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes() for _ in range(64)]
    extras = [rng.integers(0, 256, int(rng.integers(0, 33)), dtype=np.uint8).tobytes() for _ in range(64)]
    srcs = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(64)]
    dsts = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(64)]
    got = util.ipv6_checksum_many(datas, [8] * 64, extras, srcs, dsts, [6] * 64)
    for i in range(64):
        assert got[i] == coracle.ipv6_checksum(datas[i], 8, extras[i], srcs[i], dsts[i], 6)
    a4, b4 = ipaddress.IPv4Address("10.1.2.3"), ipaddress.IPv4Address("10.9.8.7")
    for i in range(0, 64, 9):
        assert udp.ipv4_checksum_adv(datas[i], extras[i], a4, b4) == \
            coracle.ipv4_checksum(datas[i], 3, extras[i], a4.packed, b4.packed, 17)
        assert tcp.ipv6_checksum_adv(datas[i], extras[i], srcs[i], dsts[i]) == \
            coracle.ipv6_checksum(datas[i], 8, extras[i], srcs[i], dsts[i], 6)
    assert util.checksum(b"", 0) == 0
