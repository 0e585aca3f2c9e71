"""GPU: the receive kernels' run scheduling (RxArgs::sched).

A launch hands each persistent wave a static grid-stride share of the batch's
runs and lets the waves claim the rest from counters: one block of the
context's pool, held by that launch alone and handed back zeroed by its last
wave. These tests check that every run is processed exactly once whatever the
static share and the counter count, across ragged batch ends, every kernel kind
that claims (small, MTU, mixed), block reuse over many launches, launches of
one context interleaved on several streams, a destroyed stream handle reused
with work in flight, more launches in flight than the pool has blocks (static
fallback), and launches captured into a HIP graph and replayed. Results are
compared with the oracle (bit-exact) and the per-launch counters with the
oracle's counts; after every test all blocks are back in the pool.
"""
import ctypes

import numpy as np
import pytest
import torch

import libpnet_amd as lp
from oracle import coracle
from tests.test_gpu_parity import NTHREADS, compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu

# big enough that the batch has at least 8 runs per resident wave (the launch's
# claim threshold) on a 256-CU MI355X: 4096 waves x 8 runs x 64 frames; the
# MTU kernel runs with 1 block per CU here (1024 waves) to keep its batch small
SIZES = {"udp64": (1 << 21) + 37, "tcp1500": (1 << 19) + 5, "imix": (1 << 21) + 11}
BLOCKS_PER_CU = {"tcp1500": "1"}


class _Dev:
    """The batch resident on the GPU (frames and descriptors), uploaded once
    and synchronized, so launches on any stream may read it."""

    def __init__(self, w):
        self.w = w
        self.d = to_dev(w.buf)
        if not w.stride:
            self.offs = to_dev(w.offsets.astype(np.int64))
            self.lens = to_dev(w.lengths.astype(np.int32))
        torch.cuda.synchronize()

    def run(self, n, stream=None, cols=lp.IPV4_COLUMNS, out=None):
        w = self.w
        if w.stride:
            return lp.rx_process(self.d, stride=w.stride, frame_len=w.frame_len, n_frames=n, columns=cols,
                                 stream=stream, out=out)
        return lp.rx_process(self.d, offsets=self.offs, lengths=self.lens, columns=cols, stream=stream, out=out)


def _outs(k, n, cols=lp.IPV4_COLUMNS):
    """k result blocks with zeroed counters, allocated and zeroed (on the
    current stream) BEFORE launches on other streams: an RxResult made per
    launch zeroes its counters on the current stream, which is not ordered
    with a launch on another stream (with 4 hardware queues a stream's zeroing
    can even queue behind another stream's held work)."""
    outs = [lp.RxResult(n, "cuda:0", cols, counters=True) for _ in range(k)]
    torch.cuda.synchronize()
    return outs


def _stats():
    return lp.engine.context(0).sched_stats()


def _delta(a, b):
    return {k: b[k] - a[k] for k in ("claimed", "static_busy", "static_captured")}


def _hip():
    # the HIP runtime already in the process (PyTorch's, which libpnetgpu.so binds to)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return hip


def _oracle(w, n):
    if w.stride:
        rec = coracle.rx_batch(w.buf, n, stride=w.stride, frame_len=w.frame_len, nthreads=NTHREADS)
        return rec, np.full(n, w.frame_len, np.uint32)
    return coracle.rx_batch(w.buf, n, offsets=w.offsets, lengths=w.lengths, nthreads=NTHREADS), w.lengths


@pytest.mark.parametrize("name", list(SIZES))
def test_every_run_once_any_static_share(name, tune):
    n = SIZES[name]
    w = lp.synth.make(name, n, seed=11, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    if name in BLOCKS_PER_CU:
        tune("blocks_per_cu", BLOCKS_PER_CU[name])
    for pct, nctr in [(100, 1), (92, 32), (50, 7), (0, 64), (0, 1), (99, 3)]:
        tune("static_pct", pct)
        tune("claim_counters", nctr)
        res = dv.run(n)
        torch.cuda.synchronize()
        compare(res, rec)
        assert res.counter_dict() == want, (pct, nctr)


def test_counter_blocks_reused_across_many_launches(tune):
    """150 launches on one stream with no host synchronization: each takes a
    free block of the pool (or runs static once all 64 are held), must start
    from zero claims, and hands its block back at the end."""
    n = SIZES["udp64"]
    w = lp.synth.make("udp64", n, seed=12, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    tune("static_pct", 90)
    tune("claim_counters", 16)
    s0 = _stats()
    results = [dv.run(n) for _ in range(150)]
    torch.cuda.synchronize()
    d = _delta(s0, _stats())
    assert d["claimed"] + d["static_busy"] == 150 and d["claimed"] >= 64, d
    for i in (0, 63, 64, 65, 127, 128, 149):
        compare(results[i], rec)
    for r in results:
        assert r.counter_dict() == want
    assert lp.engine.context(0).sched_conflicts() == 0
    assert _stats()["blocks_held"] == 0


def test_more_launches_in_flight_than_blocks(tune):
    """Four streams held behind a spin kernel: the first 64 launches take the
    pool's 64 blocks, the other 36 find every block held and run the static
    schedule (exactly so when the gate still held after the last enqueue; a
    host slower than the gate sees blocks come back, and only the totals hold). Every record equals the oracle's, and once the launches are done
    every block is back."""
    n = 8 * 1024 * 64                         # 8 runs x 256 CUs x 4 waves x 64 frames
    w = lp.synth.make("udp64", n, seed=17, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    tune("blocks_per_cu", 1)
    tune("static_pct", 25)
    streams = [torch.cuda.Stream() for _ in range(4)]
    outs = _outs(100, n, ("status", "l4_csum"))   # before the gate: _outs synchronizes
    gate_s, gate = torch.cuda.Stream(), torch.cuda.Event()
    with torch.cuda.stream(gate_s):
        torch.cuda._sleep(int(3e8))           # holds the launches until all 100 are enqueued
    gate.record(gate_s)
    for s in streams:
        s.wait_event(gate)
    s0 = _stats()
    assert s0["blocks_held"] == 0 and s0["blocks"] == 64
    results = [dv.run(n, stream=streams[i % 4], out=outs[i]) for i in range(100)]
    d = _delta(s0, _stats())
    gate_held = not gate.query()              # no launch can have finished and handed a block back
    torch.cuda.synchronize()
    assert d["claimed"] + d["static_busy"] == 100 and d["claimed"] >= 64 and d["static_captured"] == 0, d
    if gate_held:                             # a slow host can outlast the gate: then the split is not fixed
        assert d == {"claimed": 64, "static_busy": 36, "static_captured": 0}, d
    compare(results[0], rec)
    for i, r in enumerate(results):
        for c, col in r.columns.items():
            assert torch.equal(col, results[0].columns[c]), (i, c)
        assert r.counter_dict() == want, i
    assert _stats()["blocks_held"] == 0


def test_destroyed_stream_handle_reused_with_work_in_flight(tune):
    """Launches on a raw HIP stream, which is destroyed with them in flight;
    a new stream (often at the same handle) takes more launches at once. No
    launch shares counters with another, so every record is exact and rc 0
    means right."""
    n = SIZES["udp64"]
    w = lp.synth.make("udp64", n, seed=18, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    tune("static_pct", 50)
    hip = _hip()
    h1, h2 = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(h1)) == 0
    s1 = torch.cuda.ExternalStream(h1.value)
    outs = _outs(12, n)
    s0 = _stats()
    first = [dv.run(n, stream=s1, out=outs[i]) for i in range(6)]
    assert hip.hipStreamDestroy(h1) == 0
    assert hip.hipStreamCreate(ctypes.byref(h2)) == 0
    s2 = torch.cuda.ExternalStream(h2.value)
    second = [dv.run(n, stream=s2, out=outs[6 + i]) for i in range(6)]
    torch.cuda.synchronize()
    assert hip.hipStreamDestroy(h2) == 0
    assert _delta(s0, _stats())["claimed"] == 12
    for r in (first[0], first[-1], second[0], second[-1]):
        compare(r, rec)
    for r in first + second:
        assert r.counter_dict() == want
    assert _stats()["blocks_held"] == 0


def test_graph_capture_replays(tune):
    """A launch captured into a HIP graph runs the static schedule (a replay
    cannot take a fresh block): replayed three times, each replay's records and
    counters equal the oracle's; the uncaptured launch beside it claims."""
    n = SIZES["imix"]
    w = lp.synth.make("imix", n, seed=19, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    tune("static_pct", 50)
    res = lp.RxResult(n, "cuda:0", lp.IPV4_COLUMNS, counters=True)
    lp.rx_process(dv.d, offsets=dv.offs, lengths=dv.lens, out=res)   # first use outside the capture
    torch.cuda.synchronize()
    s0 = _stats()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        res.counters.zero_()
        lp.rx_process(dv.d, offsets=dv.offs, lengths=dv.lens, out=res)
    assert _delta(s0, _stats())["static_captured"] == 1
    for rep in range(3):
        res.block.fill_(0x5A)
        g.replay()
        torch.cuda.synchronize()
        compare(res, rec)
        assert res.counter_dict() == want, rep
    other = dv.run(n)
    torch.cuda.synchronize()
    compare(other, rec)
    assert _delta(s0, _stats())["claimed"] == 1
    assert _stats()["blocks_held"] == 0


def test_three_streams_no_host_sync(tune):
    """150 launches of one context spread over three streams with no host
    synchronization in between (more launches in flight than the context
    has counter slots): every stream claims from its own slot, every record
    equals the oracle and no claim saw another launch's epoch. The batch has
    exactly 8 runs per resident wave at one block per CU, so each launch
    claims runs."""
    n = 8 * 1024 * 64                         # 8 runs x 256 CUs x 4 waves x 64 frames
    w = lp.synth.make("udp64", n, seed=15, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    tune("blocks_per_cu", 1)
    tune("static_pct", 25)
    tune("claim_counters", 8)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = _outs(150, n)
    results = [dv.run(n, stream=streams[i % 3], out=outs[i]) for i in range(150)]
    torch.cuda.synchronize()
    compare(results[0], rec)
    for i, r in enumerate(results):
        for c, col in r.columns.items():              # the same records as the oracle-checked launch
            assert torch.equal(col, results[0].columns[c]), (i, c)
        assert r.counter_dict() == want, i
    assert lp.engine.context(0).sched_conflicts() == 0
    assert _stats()["blocks_held"] == 0


@pytest.mark.parametrize("pct,nctr", [(0, 64), (50, 7), (92, 1)])
def test_slice_kernels_claim_path(pct, nctr, tune):
    """The slice kernels' claimed units (slice_run_kernel's runs of 64 slices,
    slice_kernel's groups of 4, slice_strided_kernel's blocks of runs): one
    resident block per CU (1024 waves) and batches of more than 8 units per
    wave, so every launch claims; util::checksum through both descriptor
    kernels, the compact and strided entry points and ipv4_checksum_adv,
    bit-exact with the oracle at static shares 0, 50 and 92 %."""
    tune("slice_blocks_per_cu", 1)
    tune("static_pct", pct)
    tune("claim_counters", nctr)
    rng = np.random.default_rng(40 + pct)
    n = 8192 * 64 + 29                        # 8 runs of 64 slices per wave, a ragged last run
    buf = rng.integers(0, 256, 1 << 24, dtype=np.uint8)
    lens = rng.integers(0, 120, n).astype(np.uint32)
    big = rng.random(n) < 0.05
    lens[big] = rng.integers(120, 1500, int(big.sum()))
    offs = rng.integers(0, buf.size - 1600, n).astype(np.uint64)
    skips = np.where(rng.random(n) < 0.8, rng.integers(0, 30, n), rng.integers(0, 900, n)).astype(np.uint32)
    want = coracle.checksum_slices(buf, offs, lens, skips)
    d = to_dev(buf)
    do, dl, ds = to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)), to_dev(skips.astype(np.int32))
    desc = lp.slice_descriptors(offs, lens, skips, device="cuda:0")
    for kern in ("run", "group"):
        tune("slice_kernel", kern)
        got = lp.checksum_slices(d, do, dl, ds).cpu().numpy().view(np.uint16)
        assert np.array_equal(got, want), kern
        got = lp.checksum_slices_compact(d, desc).cpu().numpy().view(np.uint16)
        assert np.array_equal(got, want), ("compact", kern)
        eo = rng.integers(0, buf.size - 700, n).astype(np.uint64)
        el = rng.integers(0, 600, n).astype(np.uint32)
        addrs = rng.integers(0, 256, (n, 8), dtype=np.uint8)
        protos = rng.integers(0, 256, n, dtype=np.uint8)
        got = lp.checksum_adv_slices(4, d, do, dl, ds, to_dev(eo.astype(np.int64)), to_dev(el.astype(np.int32)),
                                     to_dev(addrs), to_dev(protos)).cpu().numpy().view(np.uint16)
        for i in list(range(0, n, 509)) + [n - 1]:
            o, ln, e0, e1 = int(offs[i]), int(lens[i]), int(eo[i]), int(el[i])
            assert got[i] == coracle.ipv4_checksum(bytes(buf[o:o + ln]), int(skips[i]), bytes(buf[e0:e0 + e1]),
                                                   bytes(addrs[i, :4]), bytes(addrs[i, 4:]), int(protos[i])), i
    tune("slice_kernel", None)
    # uniform 20-B slices: blocks of 3 runs (192 slices) per unit, 8 units per wave
    ns = 8 * 1024 * 192 + 77
    sbuf = rng.integers(0, 256, ns * 20 + 3, dtype=np.uint8)
    got = lp.checksum_slices_strided(to_dev(sbuf), ns, 20, 20, 5, first_offset=3).cpu().numpy().view(np.uint16)
    so = 3 + 20 * np.arange(ns, dtype=np.uint64)
    swant = coracle.checksum_slices(sbuf, so, np.full(ns, 20, np.uint32), np.full(ns, 5, np.uint32))
    assert np.array_equal(got, swant)
    torch.cuda.synchronize()
    assert _stats()["blocks_held"] == 0


def test_many_streams(tune):
    """70 streams (PyTorch's pool: distinct handles or not), two launches each
    with no host synchronization: every record equal to the oracle-checked
    one, whichever blocks the launches took."""
    n = 8 * 1024 * 64
    w = lp.synth.make("udp64", n, seed=16, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    tune("blocks_per_cu", 1)
    tune("static_pct", 25)
    streams = [torch.cuda.Stream() for _ in range(70)]
    outs = _outs(140, n, ("status", "l4_csum"))
    results = [dv.run(n, stream=streams[i % 70], out=outs[i]) for i in range(140)]
    torch.cuda.synchronize()
    compare(results[0], rec)
    for i, r in enumerate(results):
        for c, col in r.columns.items():
            assert torch.equal(col, results[0].columns[c]), (i, c)
        assert r.counter_dict() == want, i
    assert lp.engine.context(0).sched_conflicts() == 0
    assert _stats()["blocks_held"] == 0
