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
