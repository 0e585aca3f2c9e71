"""C oracle vs the independent Python restatement for the opt-in dispatch
extensions (VLAN/QinQ tags, IPv6 extension headers), and the extensions'
no-op property on frames without tags/extension headers."""
import numpy as np
import pytest

from oracle import coracle, pyoracle
from tests import framegen

FLAGS = [0, pyoracle.RX_VLAN, pyoracle.RX_IPV6_EXT, pyoracle.RX_VLAN | pyoracle.RX_IPV6_EXT]


@pytest.mark.parametrize("flags", FLAGS)
def test_extension_frames_c_vs_python(flags):
    frames = framegen.extension_frames(np.random.default_rng(21))
    buf, offs, lens = framegen.pack(frames, gap=5, rng=np.random.default_rng(3))
    recs = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    for i, f in enumerate(frames):
        exp = pyoracle.rx_frame(f, flags)
        for k in pyoracle.FIELDS:
            g = bytes(recs[i][k]) if k.endswith("ipv6") else int(recs[i][k])
            assert g == exp[k], (i, k, flags, f.hex())


def test_extensions_are_noop_without_tags():
    frames = framegen.random_frames(np.random.default_rng(5), 500)
    buf, offs, lens = framegen.pack(frames)
    a = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=0)
    b = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=3)
    # random frames carry no VLAN TPID / extension next-headers except by chance
    same = (a == b)
    assert same.mean() > 0.97


def test_vlan_and_ext_checksums_verify():
    rng = np.random.default_rng(8)
    f = framegen.add_vlan(framegen.ipv6_with_ext(rng, [0, 60, 43], "udp", 100), [(0x88A8, 3), (0x8100, 4)])
    r = coracle.rx_frame(f, 3)
    assert r["status"] & pyoracle.ST_VLAN and r["status"] & pyoracle.ST_L4_CSUM_OK
    assert r["l3_offset"] == 22 and r["ip_proto"] == 17 and r["vlan_tci"] == 3
    r0 = coracle.rx_frame(f, 0)
    assert r0["status"] == pyoracle.ST_UNKNOWN_ETHERTYPE and r0["ethertype"] == 0x88A8


def ip_packets(rng, n=600):
    """Layer-3 buffers (pnet_transport Layer3 receive): the framegen frames
    without their Ethernet header, plus short / garbage / other-version ones."""
    frames = framegen.extension_frames(rng) + framegen.random_frames(rng, n) + framegen.edge_frames(rng)
    out = [f[14:] for f in frames if len(f) >= 14]
    for k in range(40):
        out.append(bytes([(k % 16) << 4 | 5]) + rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8).tobytes())
    out += [b"", b"\x45", b"\x60" * 39]
    return out


@pytest.mark.parametrize("flags", [pyoracle.RX_L3, pyoracle.RX_L3 | pyoracle.RX_IPV6_EXT,
                                   pyoracle.RX_L3 | pyoracle.RX_VLAN | pyoracle.RX_IPV6_EXT])
def test_l3_packets_c_vs_python(flags):
    pkts = ip_packets(np.random.default_rng(31))
    buf, offs, lens = framegen.pack(pkts, gap=3, rng=np.random.default_rng(4))
    recs = coracle.rx_batch(buf, len(pkts), offsets=offs, lengths=lens, flags=flags)
    for i, f in enumerate(pkts):
        exp = pyoracle.rx_frame(f, flags)
        for k in pyoracle.FIELDS:
            g = bytes(recs[i][k]) if k.endswith("ipv6") else int(recs[i][k])
            assert g == exp[k], (i, k, flags, f.hex())


@pytest.mark.parametrize("ext", [0, pyoracle.RX_IPV6_EXT])
def test_l3_mode_equals_ethernet_mode_shifted(ext):
    """An IP packet seen at layer 3 gives the Ethernet chain's record for the same
    packet behind a 14-B Ethernet header, with every frame offset 14 lower (and
    no Ethernet view: the MAC columns are 0)."""
    rng = np.random.default_rng(32)
    frames = framegen.random_frames(rng, 800) + framegen.edge_frames(rng) + framegen.extension_frames(rng)
    n = 0
    for f in frames:
        if len(f) < 15:
            continue
        et, ver = (f[12] << 8) | f[13], f[14] >> 4
        if (et, ver) not in ((0x0800, 4), (0x86DD, 6)):
            continue
        a, b = pyoracle.rx_frame(f, ext), pyoracle.rx_frame(f[14:], ext | pyoracle.RX_L3)
        assert b["l3_offset"] == 0 and a["l3_offset"] == 14
        assert b["l4_offset"] == (a["l4_offset"] - 14 if a["l4_offset"] else 0)
        assert b["eth_dst"] == b["eth_src"] == 0
        for k in pyoracle.FIELDS:
            if k not in ("l3_offset", "l4_offset", "eth_dst", "eth_src"):
                assert a[k] == b[k], (k, f.hex())
        n += 1
    assert n > 400


def test_l3_mode_version_dispatch():
    assert pyoracle.rx_frame(b"", pyoracle.RX_L3)["status"] == pyoracle.ST_UNKNOWN_ETHERTYPE
    r = pyoracle.rx_frame(b"\x45" + bytes(10), pyoracle.RX_L3)
    assert r["status"] == pyoracle.ST_L3_IPV4 | pyoracle.ST_L3_MALFORMED and r["ethertype"] == 0x0800
    r = pyoracle.rx_frame(b"\x55" + bytes(40), pyoracle.RX_L3)
    assert r["status"] == pyoracle.ST_UNKNOWN_ETHERTYPE and r["ethertype"] == 0


def test_icmp_sequence_only_for_echo_types():
    """icmp_sequence is the echo views' get_sequence_number: set for ICMP 0/8 and
    ICMPv6 128/129 with >= 8 B, 0 for every other type (a Destination
    Unreachable's bytes 6-7 are not a sequence number); both restatements agree."""
    frames, echo = framegen.icmp_type_frames(np.random.default_rng(9))
    for f, e in zip(frames, echo):
        rc = coracle.rx_frame(f)
        rp = pyoracle.rx_frame(f)
        l4 = int(rc["l4_offset"])
        seq = (f[l4 + 6] << 8 | f[l4 + 7]) if e else 0
        assert int(rc["icmp_sequence"]) == seq == int(rp["icmp_sequence"]), (f[l4], len(f) - l4)
        assert rc["status"] & pyoracle.ST_L4_CSUM_OK
