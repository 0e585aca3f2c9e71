"""GPU parity of the mixed shape's large-frame runs (rx_generic.h, kUniRuns):
a run of 64 frames whose every frame is at least 768 B (and under 4 KiB) is
streamed in the MTU shape's unified order inside the mixed kernel, and a run of
frames all at least 4 KiB with the jumbo shape's tail (descriptor batches
without a size hint). Bursts of such runs between mixed runs, at any alignment, with and
without the parse extensions, the header-field columns and TX; runs that just
miss the bar (one 767-B frame, one invalid descriptor); and the bench's
no-hint 1500-B descriptor batch at full size — every column and counter equal
to the oracle (the reference's receive chain, packetdump.rs:120-217)."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import NTHREADS, compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu


def bursty_frames(rng, nruns):
    """Runs of 64 frames: large-only (768..3000 B), mixed, large with one
    frame just under the bar, jumbo-only (>= 4096 B), and 4095-B frames with
    one 4096-B frame."""
    frames = []
    for r in range(nruns):
        kind = r % 6
        if kind in (0, 1):
            frames += framegen.random_frames(rng, 64, min_len=768, max_len=3000)
        elif kind == 2:
            frames += framegen.random_frames(rng, 64, max_len=1600)
        elif kind == 3:
            run = framegen.random_frames(rng, 64, min_len=768, max_len=1600)
            run[int(rng.integers(0, 64))] = framegen.random_frames(rng, 1, min_len=767, max_len=767)[0]
            frames += run
        elif kind == 4:                         # jumbo run (every frame >= 4096 B)
            frames += framegen.random_frames(rng, 64, min_len=4096, max_len=9100)
        else:                                   # large run with one frame at the jumbo bar
            run = framegen.random_frames(rng, 64, min_len=4095, max_len=4095)
            run[int(rng.integers(0, 64))] = framegen.random_frames(rng, 1, min_len=4096, max_len=4096)[0]
            frames += run
    return frames


def run_batch(buf, offs, lens, flags=0, columns=ALL_COLUMNS, compact=True, data_offset=0):
    d = to_dev(np.concatenate([np.zeros(16, np.uint8), buf]))[data_offset:]
    offs = offs + 16 - data_offset
    if compact:
        o, ln = to_dev(np.asarray(offs, np.uint32).view(np.int32)), to_dev(np.asarray(lens, np.uint16).view(np.int16))
        flags |= lp.DESC_COMPACT
    else:
        o, ln = to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32))
    res = lp.rx_process(d, offsets=o, lengths=ln, columns=columns, flags=flags, counters=True)
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("flags", [0, 3])
@pytest.mark.parametrize("columns", ["ipv4", "all"])
def test_bursts_of_large_runs(flags, columns):
    rng = np.random.default_rng(80 + flags)
    frames = bursty_frames(rng, 96)
    buf, offs, lens = framegen.pack(frames, gap=int(rng.integers(0, 9)), rng=rng)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    cols = lp.IPV4_COLUMNS if columns == "ipv4" else ALL_COLUMNS
    for data_offset, compact in ((0, True), (5, True), (3, False)):
        res = run_batch(buf, offs, lens, flags=flags, columns=cols, compact=compact, data_offset=data_offset)
        compare(res, rec)
        assert res.counter_dict() == oracle_counters(rec, lens)


def test_large_runs_with_an_invalid_descriptor_and_a_short_last_run():
    """A large run with one descriptor past the buffer (that run stays in the
    window-first order) and a batch ending in a partial large run."""
    rng = np.random.default_rng(88)
    frames = framegen.random_frames(rng, 64 * 5 + 17, min_len=768, max_len=2000)
    buf, offs, lens = framegen.pack(frames, gap=3, rng=rng)
    offs, lens = offs.astype(np.uint64).copy(), lens.astype(np.uint32).copy()
    offs[70], lens[70] = buf.size + 100, 1000
    lens[200] = buf.size                    # runs past the end
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
    assert rec["status"][70] & 0x8000 and rec["status"][200] & 0x8000
    res = run_batch(buf, offs, lens, compact=False)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


def test_tx_fill_bursts_of_large_runs():
    rng = np.random.default_rng(89)
    frames = bursty_frames(rng, 40)
    buf, offs, lens = framegen.pack(frames, gap=2, rng=rng)
    want_buf, want_rec = coracle.tx_fill(buf, len(offs), offsets=offs, lengths=lens)
    d = to_dev(buf)
    res = lp.tx_fill_checksums(d, offsets=to_dev(np.asarray(offs, np.uint32).view(np.int32)),
                               lengths=to_dev(np.asarray(lens, np.uint16).view(np.int16)), columns=ALL_COLUMNS,
                               flags=lp.DESC_COMPACT)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), want_buf)
    compare(res, want_rec)


@pytest.mark.parametrize("name,n", [("udp1500", 1 << 20), ("udp6_jumbo", 1 << 17)])
def test_descriptor_batch_without_hint_full_size(name, n):
    """bench.py's descriptor line (`descriptor.no_hint`): the 2^20-frame 1500-B
    UDP batch (and the 9000-B jumbo batch) as compact descriptors with no size
    hint — the mixed kernel, every run large — against the oracle, planted
    corruptions included."""
    w = lp.synth.make(name, n, seed=1000, corrupt_ppm=10000)
    offs = np.arange(w.n, dtype=np.uint64) * np.uint64(w.stride)
    lens = np.full(w.n, w.frame_len, np.uint32)
    rec = coracle.rx_batch(w.buf, w.n, offsets=offs, lengths=lens, nthreads=NTHREADS)
    res = lp.rx_process(to_dev(w.buf), offsets=to_dev(offs.astype(np.uint32).view(np.int32)),
                        lengths=to_dev(lens.astype(np.uint16).view(np.int16)), columns=lp.IPV4_COLUMNS,
                        flags=lp.DESC_COMPACT, counters=True)
    torch.cuda.synchronize()
    assert "rx_kernel<8, 4, 8" in lp.last_rx_kernel()      # the mixed shape took it
    compare(res, rec)
    c = res.counter_dict()
    assert c == oracle_counters(rec, lens)
    assert c["ip_csum_bad"] == w.expect["ip_bad"] and c["l4_csum_bad"] == w.expect["l4_bad"]
