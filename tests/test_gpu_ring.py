"""GPU end-to-end of the batch producer: frames pushed one by one (or from a pcap
replay) through the pinned ring come back with records identical to the oracle's."""
import numpy as np
import pytest

import libpnet_amd as lp
from oracle import coracle
from tests import framegen
from tests.pcaputil import write_pcap

pytestmark = pytest.mark.gpu


def check_batches(batches, frames):
    got = sorted(batches, key=lambda b: b.id)
    assert [b.id for b in got] == list(range(len(got)))
    assert sum(b.n for b in got) == len(frames)
    i = 0
    for b in got:
        for k in range(b.n):
            assert bytes(b.frames[b.offsets[k]:b.offsets[k] + b.lengths[k]]) == frames[i + k]
        rec = coracle.rx_batch(b.frames, b.n, offsets=b.offsets, lengths=b.lengths)
        for c, v in b.records.items():
            assert np.array_equal(v, rec[c]), (b.id, c)
        i += b.n


def test_ring_pcap_replay(tmp_path):
    rng = np.random.default_rng(9)
    frames = framegen.edge_frames(rng) + framegen.random_frames(rng, 4000, max_len=9000)
    p = tmp_path / "replay.pcap"
    write_pcap(p, frames)
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=700)     # many small batches: every slot state
    out = []
    for f in lp.pcap_frames(p):
        out.extend(ring.feed(f))
    out.extend(ring.drain())
    check_batches(out, frames)


def test_ring_feed_many_synth():
    w = lp.synth.make("imix", 50000, seed=6)
    frames = [bytes(w.buf[o:o + l]) for o, l in zip(w.offsets, w.lengths)]
    ring = lp.Ring(batch_bytes=4 << 20, batch_frames=1 << 14)
    out = list(ring.feed_many(w.buf, w.offsets, w.lengths)) + list(ring.drain())
    check_batches(out, frames)
    assert sum(b.counters["l4_csum_bad"] for b in out) == w.expect["l4_bad"]
