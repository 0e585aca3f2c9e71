"""GPU parity of compact descriptors (PNETGPU_DESC_COMPACT: u32 offsets, u16
lengths — SURVEY.md §8(b)'s suggested layout) vs the oracle and vs the full
u64/u32 descriptors of the same batch: random and extension frames at any
alignment (with and without the parse extensions), invalid descriptors, the
full-size IMIX workload against the oracle, and the pinned ring, which ships compact descriptors
whenever a batch qualifies."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import NTHREADS, compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu


def run_compact(d, offs, lens, flags=0, columns=ALL_COLUMNS):
    res = lp.rx_process(d, offsets=to_dev(np.asarray(offs, np.uint32).view(np.int32)),
                        lengths=to_dev(np.asarray(lens, np.uint16).view(np.int16)), columns=columns,
                        flags=flags | lp.DESC_COMPACT)
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("flags", [0, 3])
def test_compact_random_and_extension_frames(flags):
    rng = np.random.default_rng(70 + flags)
    frames = framegen.extension_frames(rng) + framegen.random_frames(rng, 4000, max_len=9100)
    buf, offs, lens = framegen.pack(frames, gap=13, rng=rng)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    for data_offset in (0, 5):
        d = to_dev(np.concatenate([np.zeros(16, np.uint8), buf]))[data_offset:]
        res = run_compact(d, offs + 16 - data_offset, lens, flags=flags)
        compare(res, rec)
        assert res.counter_dict() == oracle_counters(rec, lens)


def test_compact_invalid_descriptors():
    """Offsets past the end (up to 2^32 - 1) and lengths running past it are
    flagged DESC_INVALID, exactly as with full descriptors."""
    rng = np.random.default_rng(9)
    frames = framegen.random_frames(rng, 400)
    buf, offs, lens = framegen.pack(frames)
    offs = offs.astype(np.uint64).copy()
    lens = lens.astype(np.uint32).copy()
    size = buf.size
    for k, (o, n) in enumerate([(size, 64), (size + 1, 14), (2**32 - 1, 60), (2**31, 1), (size - 10, 11),
                                (size - 100, 65535), (size - 20, 20)]):
        offs[k], lens[k] = o, n
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
    assert (rec["status"][:6] & 0x8000).all() and not rec["status"][6] & 0x8000
    res = run_compact(to_dev(buf), offs, lens)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


def test_compact_imix_full_size_vs_oracle():
    """The bench's IMIX form (configs[3]: compact descriptors, 2^22 frames per
    GPU, 1 % planted corruptions) against the oracle directly: every record
    column, the counters, and every planted corruption found — the very batch
    `python bench.py` times at N = 1 (its default --seed 1: synth seed 1000)."""
    w = lp.synth.make("imix", 1 << 22, seed=1000, corrupt_ppm=10000)
    rec = coracle.rx_batch(w.buf, w.n, offsets=w.offsets, lengths=w.lengths, nthreads=NTHREADS)
    comp = run_compact(to_dev(w.buf), w.offsets, w.lengths, columns=lp.IPV4_COLUMNS)
    compare(comp, rec)
    c = comp.counter_dict()
    assert c == oracle_counters(rec, w.lengths)
    assert c["frames"] == 1 << 22
    assert c["ip_csum_bad"] == w.expect["ip_bad"] and c["l4_csum_bad"] == w.expect["l4_bad"]


def test_ring_ships_compact_descriptors_and_full_ones_for_long_frames():
    """The ring's batches (compact when every frame < 64 KiB, full otherwise)
    equal the oracle; a 70,000-B frame forces the full form for its batch."""
    rng = np.random.default_rng(21)
    frames = framegen.random_frames(rng, 3000, max_len=1600)
    big = bytearray(framegen.build_frame(rng, "udp", 100))
    big += bytes(70000 - len(big))
    frames.insert(1500, bytes(big))
    buf, offs, lens = framegen.pack(frames, gap=5, rng=rng)
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=1000, columns=ALL_COLUMNS)   # copy=True: batches outlive waits
    try:
        got = list(ring.feed_region(buf, offs, lens)) + list(ring.drain())
    finally:
        ring.close()
    assert [b.id for b in got] == list(range(len(got))) and len(got) >= 4
    assert sum(b.n for b in got) == len(offs)
    for c in ALL_COLUMNS:
        assert np.array_equal(np.concatenate([b.records[c] for b in got]), rec[c]), c


def test_compact_any_order_overlaps_empty_and_max_length():
    """Compact descriptor batches the mixed kernel must take: frames in shuffled
    order, frames that overlap other frames, zero-length frames, and 65535-B
    frames (the compact maximum) at every alignment — every column equal to the
    oracle."""
    rng = np.random.default_rng(404)
    frames = framegen.random_frames(rng, 3000, max_len=3000) + framegen.edge_frames(rng)
    buf, offs, lens = framegen.pack(frames, gap=7, rng=rng)
    offs, lens = offs.astype(np.uint64), lens.astype(np.uint32)
    big = rng.integers(0, 256, 70000, dtype=np.uint8)
    big[12:14] = (8, 0)
    big[14] = 0x45
    base = buf.size
    buf = np.concatenate([buf, big, np.zeros(32, np.uint8)])
    extra_o = [base + a for a in (0, 1, 7, 15, 16, 4000)] + [int(o) + 3 for o in offs[:200:7]] + [5, 9, base]
    extra_l = [65535, 65535, 65535, 65535, 60000, 65535 - 4000] + [max(0, int(l) - 5) for l in lens[:200:7]] + [0, 0, 0]
    offs = np.concatenate([offs, np.array(extra_o, np.uint64)])
    lens = np.concatenate([lens, np.array(extra_l, np.uint32)])
    perm = rng.permutation(len(offs))
    offs, lens = offs[perm], lens[perm]
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
    res = run_compact(to_dev(buf), offs, lens)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


def test_compact_tx_fill_equals_oracle():
    """tx_fill_checksums over compact descriptors: patched bytes and pre-patch
    records equal oracle_tx_fill."""
    rng = np.random.default_rng(405)
    frames = framegen.random_frames(rng, 4000, max_len=1600)
    buf, offs, lens = framegen.pack(frames, gap=3, rng=rng)
    want_buf, want_rec = coracle.tx_fill(buf, len(offs), offsets=offs, lengths=lens)
    d = to_dev(buf)
    res = lp.tx_fill_checksums(d, offsets=to_dev(np.asarray(offs, np.uint32).view(np.int32)),
                               lengths=to_dev(np.asarray(lens, np.uint16).view(np.int16)), columns=ALL_COLUMNS,
                               flags=lp.DESC_COMPACT)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), want_buf)
    compare(res, want_rec)
