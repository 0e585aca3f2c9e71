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
