"""GPU parity of rx_small_dma_kernel (the small kernel's batches with frames
staged by LDS-DMA, the PNETGPU_TUNE_SMALL_DMA kernel) against the oracle:
every stride / frame length / first offset the small kernel takes, ragged
batch ends (the DMA of lanes past the batch), steered random bytes through its
register fast path and generic fallback, both record forms at full per-GPU
size, claimed run schedules, and many launches over three streams."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import NTHREADS, compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu
DMA_KERNEL = "rx_small_dma_kernel<3>"
# every record column the DMA kernel writes (no IPv6 addresses: they need the linear slot)
DMA_COLUMNS = tuple(c for c in lp.RECORD_COLUMNS if c not in ("src_ipv6", "dst_ipv6"))
VERIFY = ("status", "ip_csum", "l4_csum")


@pytest.fixture
def dma(tune):
    tune("small_dma", 1)
    return tune


@pytest.mark.parametrize("stride", [16, 48, 64, 80, 128])
def test_dma_strides_and_lengths(stride, dma):
    rng = np.random.default_rng(500 + stride)
    n = 64 * 37 + 29                                   # a ragged last run
    kinds = ("udp", "tcp", "icmp", "udp6", "tcp6", "icmp6", "icmp_over6")
    frames = []
    for i in range(n):
        ihl = 5 if i % 5 else int(rng.integers(5, 16))
        f = bytearray(framegen.build_frame(rng, kinds[i % len(kinds)], int(rng.integers(0, 40)), ihl=ihl))
        if i % 9 == 0 and len(f) > 20:
            f[int(rng.integers(14, len(f)))] ^= 0x5A
        frames.append(bytes(f))
    for first in (0, 32):
        for flen in sorted({1, 13, 14, 33, 34, 41, 42, 47, 48, 53, 54, 61, 64, min(stride, 64)}):
            if flen > stride:
                continue
            buf = rng.integers(0, 256, first + stride * n + 64, dtype=np.uint8)
            for i, f in enumerate(frames):
                f = np.frombuffer(f, np.uint8)[:stride]
                buf[first + i * stride:first + i * stride + len(f)] = f
            rec = coracle.rx_batch(buf, n, first=first, stride=stride, frame_len=flen, nthreads=NTHREADS)
            # the batch ends exactly at the last frame's end: no slack after it
            d = to_dev(buf)[:first + stride * (n - 1) + flen]
            res = lp.rx_process(d, stride=stride, frame_len=flen, first_offset=first, n_frames=n, columns=DMA_COLUMNS)
            torch.cuda.synchronize()
            assert lp.last_rx_kernel() == DMA_KERNEL
            compare(res, rec)
            assert res.counter_dict() == oracle_counters(rec, np.full(n, flen, np.uint32)), (first, flen)


@pytest.mark.parametrize("frame_len", [14, 20, 34, 42, 47, 60, 64])
def test_dma_fuzz(frame_len, dma):
    rng = np.random.default_rng(3100 + frame_len)
    n = (1 << 17) + 5
    buf = rng.integers(0, 256, n * 64 + 64, dtype=np.uint8)
    f = buf[: n * 64].reshape(n, 64)
    r = rng.random(n)
    f[r < 0.7, 12], f[r < 0.7, 13] = 0x08, 0x00
    f[(r >= 0.7) & (r < 0.85), 12], f[(r >= 0.7) & (r < 0.85), 13] = 0x86, 0xDD
    f[r < 0.7, 14] = 0x40 | rng.integers(0, 16, int((r < 0.7).sum())).astype(np.uint8)
    f[r < 0.5, 14] = 0x45
    f[:, 23] = np.array([6, 17, 1, 58, 47], np.uint8)[rng.integers(0, 5, n)]
    short_tl = rng.random(n) < 0.3
    f[short_tl, 16] = 0
    f[short_tl, 17] = rng.integers(0, 64, int(short_tl.sum())).astype(np.uint8)
    rec = coracle.rx_batch(buf, n, stride=64, frame_len=frame_len, nthreads=16)
    for cols in (DMA_COLUMNS, VERIFY, ("status",)):
        res = lp.rx_process(to_dev(buf), stride=64, frame_len=frame_len, n_frames=n, columns=cols)
        torch.cuda.synchronize()
        assert lp.last_rx_kernel() == DMA_KERNEL
        compare(res, rec)


@pytest.mark.parametrize("cols", [lp.IPV4_COLUMNS, VERIFY])
def test_dma_full_size(cols, dma):
    """configs[1] at full per-GPU size (2^24 frames, 1 % planted corruptions)."""
    n = 1 << 24
    w = lp.synth.make("udp64", n, seed=3, corrupt_ppm=10000)
    res = lp.rx_process(to_dev(w.buf), stride=64, frame_len=64, n_frames=n, columns=cols)
    rec = coracle.rx_batch(w.buf, n, stride=64, frame_len=64, nthreads=NTHREADS)
    torch.cuda.synchronize()
    assert lp.last_rx_kernel() == DMA_KERNEL
    compare(res, rec)
    c = res.counter_dict()
    assert c == oracle_counters(rec, np.full(n, 64, np.uint32))
    assert c["ip_csum_bad"] == w.expect["ip_bad"] and c["l4_csum_bad"] == w.expect["l4_bad"]


def test_dma_claimed_schedules_and_three_streams(dma):
    """Every run once at static shares 0-100 % with 1-64 claim counters, then
    90 launches over three streams with no host synchronization, each equal to
    the oracle-checked one."""
    n = (1 << 21) + 37
    w = lp.synth.make("udp64", n, seed=11, corrupt_ppm=10000)
    rec = coracle.rx_batch(w.buf, n, stride=64, frame_len=64, nthreads=NTHREADS)
    want = oracle_counters(rec, np.full(n, 64, np.uint32))
    d = to_dev(w.buf)
    torch.cuda.synchronize()
    for pct, nctr in [(100, 1), (92, 32), (50, 7), (0, 64), (0, 1)]:
        dma("static_pct", pct)
        dma("claim_counters", nctr)
        res = lp.rx_process(d, stride=64, frame_len=64, n_frames=n)
        torch.cuda.synchronize()
        compare(res, rec)
        assert res.counter_dict() == want, (pct, nctr)
    dma("static_pct", 50)
    streams = [torch.cuda.Stream() for _ in range(3)]
    results = [lp.rx_process(d, stride=64, frame_len=64, n_frames=n, stream=streams[i % 3]) for i in range(90)]
    torch.cuda.synchronize()
    compare(results[0], rec)
    for i, r in enumerate(results):
        for c, col in r.columns.items():
            assert torch.equal(col, results[0].columns[c]), (i, c)
        assert r.counter_dict() == want, i
    assert lp.engine.context(0).sched_conflicts() == 0


def test_dma_not_taken_where_it_cannot_serve(dma):
    """TX, header-field and IPv6-address columns, and frame_len 0, stay on the
    register kernel (the DMA slot keeps its rotated layout)."""
    w = lp.synth.make("udp64", 4096, seed=3)
    d = to_dev(w.buf)
    lp.rx_process(d, stride=64, frame_len=64, n_frames=4096)
    assert lp.last_rx_kernel() == DMA_KERNEL
    for kw in ({"columns": ("status", "tcp_flags")}, {"columns": ("status", "src_ipv6")}, {"frame_len": 0}):
        args = {"stride": 64, "frame_len": 64, "n_frames": 4096, **kw}
        lp.rx_process(d, **args)
        assert lp.last_rx_kernel().startswith("rx_small_kernel<"), kw
    lp.tx_fill_checksums(d, stride=64, frame_len=64, n_frames=4096)
    assert lp.last_rx_kernel() == "rx_small_kernel<true, false>"
    torch.cuda.synchronize()
