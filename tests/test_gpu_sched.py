"""GPU: the receive kernels' run scheduling (RxArgs::sched).

A launch hands each persistent wave a static grid-stride share of the batch's
runs and lets the waves claim the rest from per-launch counters. These tests
check that every run is processed exactly once whatever the static share and
the counter count, across ragged batch ends, every kernel kind that claims
(small, MTU, mixed), counter-slot reuse over many launches (epochs), and
launches of one context interleaved on two streams. Results are compared with
the oracle (bit-exact) and the per-launch counters with the oracle's counts.
"""
import os

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

    def run(self, n, stream=None, cols=lp.IPV4_COLUMNS):
        w = self.w
        if w.stride:
            return lp.rx_process(self.d, stride=w.stride, frame_len=w.frame_len, n_frames=n, columns=cols,
                                 stream=stream)
        return lp.rx_process(self.d, offsets=self.offs, lengths=self.lens, columns=cols, stream=stream)


def _oracle(w, n):
    if w.stride:
        rec = coracle.rx_batch(w.buf, n, stride=w.stride, frame_len=w.frame_len, nthreads=NTHREADS)
        return rec, np.full(n, w.frame_len, np.uint32)
    return coracle.rx_batch(w.buf, n, offsets=w.offsets, lengths=w.lengths, nthreads=NTHREADS), w.lengths


@pytest.fixture
def sched_env():
    keys = ("PNETGPU_STATIC_PCT", "PNETGPU_CLAIM_COUNTERS", "PNETGPU_BLOCKS_PER_CU")
    old = {k: os.environ.get(k) for k in keys}

    def set_(pct, nctr):
        os.environ["PNETGPU_STATIC_PCT"] = str(pct)
        os.environ["PNETGPU_CLAIM_COUNTERS"] = str(nctr)
    yield set_
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("name", list(SIZES))
def test_every_run_once_any_static_share(name, sched_env):
    n = SIZES[name]
    w = lp.synth.make(name, n, seed=11, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    if name in BLOCKS_PER_CU:
        os.environ["PNETGPU_BLOCKS_PER_CU"] = BLOCKS_PER_CU[name]
    for pct, nctr in [(100, 1), (92, 32), (50, 7), (0, 64), (0, 1), (99, 3)]:
        sched_env(pct, nctr)
        res = dv.run(n)
        torch.cuda.synchronize()
        compare(res, rec)
        assert res.counter_dict() == want, (pct, nctr)


def test_counter_slots_reused_across_many_launches(sched_env):
    """More launches than the context has counter slots: each slot is taken
    again by a later epoch and must start from zero claims for it."""
    n = SIZES["udp64"]
    w = lp.synth.make("udp64", n, seed=12, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    sched_env(90, 16)
    results = [dv.run(n) for _ in range(150)]
    torch.cuda.synchronize()
    for i in (0, 63, 64, 65, 127, 128, 149):
        compare(results[i], rec)
    for r in results:
        assert r.counter_dict() == want


def test_two_streams_one_context(sched_env):
    """Launches of one context on two streams in flight together use distinct
    counter slots (one per epoch)."""
    n = SIZES["imix"]
    w = lp.synth.make("imix", n, seed=13, corrupt_ppm=10000)
    rec, lens = _oracle(w, n)
    want = oracle_counters(rec, lens)
    dv = _Dev(w)
    sched_env(80, 32)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    results = []
    for i in range(40):
        results.append(dv.run(n, stream=s1 if i % 2 else s2))
    torch.cuda.synchronize()
    for r in results:
        assert r.counter_dict() == want
    compare(results[-1], rec)
    compare(results[-2], rec)
