"""Cross-checks the C oracle against the independent Python restatement on
seeded random and edge-case frames (both restate the reference; see oracle/)."""
import numpy as np
import pytest

from oracle import coracle, pyoracle
from tests import framegen


def _compare(frames):
    buf, offs, lens = framegen.pack(frames, gap=3, rng=np.random.default_rng(1))
    recs = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens)
    for i, f in enumerate(frames):
        exp = pyoracle.rx_frame(f)
        got = recs[i]
        for k in pyoracle.FIELDS:
            g = bytes(got[k]) if k.endswith("ipv6") else int(got[k])
            assert g == exp[k], (i, k, f.hex())


def test_edge_frames():
    _compare(framegen.edge_frames(np.random.default_rng(7)))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_frames(seed):
    _compare(framegen.random_frames(np.random.default_rng(seed), 400))


def test_batch_threads_and_invalid_desc():
    rng = np.random.default_rng(3)
    frames = framegen.random_frames(rng, 300)
    buf, offs, lens = framegen.pack(frames)
    a = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, nthreads=1)
    b = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, nthreads=5)
    assert (a == b).all()
    offs2 = offs.copy()
    offs2[5] = buf.size + 1
    c = coracle.rx_batch(buf, len(frames), offsets=offs2, lengths=lens)
    assert c["status"][5] == pyoracle.ST_DESC_INVALID


def test_checksum_adv_extra_data():
    """util::ipv4/ipv6_checksum with non-empty extra_data (the udp|tcp
    *_checksum_adv wrappers, udp.rs:45-56, tcp.rs:250-261): C vs Python, and the
    odd-length quirk of util.rs:114 — the extra's trailing byte never enters the
    sum, but it does count in the pseudo-header length."""
    rng = np.random.default_rng(11)
    for alen, cfn in ((4, coracle.ipv4_checksum), (16, coracle.ipv6_checksum)):
        for _ in range(300):
            d = rng.integers(0, 256, int(rng.integers(0, 90)), dtype=np.uint8).tobytes()
            e = rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
            src = rng.integers(0, 256, alen, dtype=np.uint8).tobytes()
            dst = rng.integers(0, 256, alen, dtype=np.uint8).tobytes()
            skip, proto = int(rng.integers(0, 50)), int(rng.integers(0, 256))
            want = pyoracle.ipv4_checksum(d, skip, e, src, dst, proto)
            assert cfn(d, skip, e, src, dst, proto) == want
            if len(e) % 2:
                flipped = e[:-1] + bytes([e[-1] ^ 0xFF])
                assert cfn(d, skip, flipped, src, dst, proto) == want


def test_long_slices_wrap_like_a_release_build():
    """Slices long enough for the reference's u32 sums to wrap (util.rs:158-181,
    103-114: `sum += ...`, modulo 2^32 in a release build): both restatements
    wrap the same way — the GPU long-slice path is checked against this."""
    rng = np.random.default_rng(5)
    for ln in (131070, 131071, 131072, 200001, 1 << 20):
        for fill in (b"\xff", None):
            d = fill * ln if fill else rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
            for skip in (0, 7, ln // 2, 1 << 30):
                assert coracle.checksum(d, skip) == pyoracle.checksum(d, skip)
            src, dst = b"\xff" * 16, bytes(range(16))
            extra = d[: 70001]
            assert coracle.ipv6_checksum(d, 3, extra, src, dst, 17) == pyoracle.ipv6_checksum(d, 3, extra, src, dst, 17)
            assert coracle.ipv4_checksum(d, 3, extra, src[:4], dst[:4], 6) == \
                pyoracle.ipv4_checksum(d, 3, extra, src[:4], dst[:4], 6)
    # all 0xFF words: the exact sum passes 2^32 first at 65538 words (the wrap changes the result)
    d = b"\xff" * 131076
    exact = 65538 * 0xFFFF
    s = exact & 0xFFFFFFFF
    while s >> 16:
        s = (s >> 16) + (s & 0xFFFF)
    assert coracle.checksum(d, 1 << 30) == (~s) & 0xFFFF
