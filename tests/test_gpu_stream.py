"""GPU parity of the LDS-DMA stream kernel (rx_stream_kernel: fixed stride >= 1 KiB,
frame_len in [7/8 stride, stride]) vs the CPU oracle: random strides and lengths,
every first-offset and data-pointer alignment, run counts that end mid-run, a
buffer that ends at the last frame, the opt-in VLAN / IPv6 extension dispatch,
and the same batch through the per-frame kernel (PNETGPU_RX_KIND=2) as a cross-check.
The stream kernel is selected with PNETGPU_RX_KIND=4 (it is not the default yet)."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import NTHREADS, compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def stream_kind(monkeypatch):
    monkeypatch.setenv("PNETGPU_RX_KIND", "4")


def stride_batch(rng, frames, stride, first, tail=64):
    buf = rng.integers(0, 256, first + stride * len(frames) + tail, dtype=np.uint8)
    for i, f in enumerate(frames):
        f = np.frombuffer(f, np.uint8)[:stride]
        buf[first + i * stride:first + i * stride + len(f)] = f
    return buf


@pytest.mark.parametrize("seed", range(6))
def test_stream_random_geometry(seed, monkeypatch):
    rng = np.random.default_rng(900 + seed)
    stride = int(rng.integers(1024, 9200))
    flen = int(rng.integers(-(-7 * stride // 8), stride + 1))
    n = int(rng.choice([1, 63, 64, 65, 129, 200 + seed * 37]))
    first = int(rng.integers(0, 40))
    data_offset = int(rng.integers(0, 16))
    frames = framegen.random_frames(rng, n, min_len=flen - 200, max_len=flen + 64)
    buf = stride_batch(rng, frames, stride, first + data_offset)
    rec = coracle.rx_batch(buf[data_offset:], n, first=first, stride=stride, frame_len=flen, nthreads=NTHREADS)
    d = to_dev(buf)[data_offset:]
    for kind in ("4", "2"):
        monkeypatch.setenv("PNETGPU_RX_KIND", kind)
        res = lp.rx_process(d, stride=stride, frame_len=flen, first_offset=first, n_frames=n, columns=ALL_COLUMNS)
        torch.cuda.synchronize()
        compare(res, rec)
        assert res.counter_dict() == oracle_counters(rec, np.full(n, flen, np.uint32)), (stride, flen, n, kind)


@pytest.mark.parametrize("stride,flen", [(1024, 1024), (1500, 1500), (1514, 1325), (9018, 9018)])
def test_stream_buffer_ends_at_last_frame(stride, flen):
    """data_bytes ends exactly at the last frame's end (the kernel clamps its
    granule loads to the last readable 16 B)."""
    rng = np.random.default_rng(stride)
    n = 130
    frames = [framegen.build_frame(rng, k, flen - 54) for k in ("udp", "tcp") * (n // 2)]
    buf = stride_batch(rng, frames, stride, 0, tail=0)
    end = (n - 1) * stride + flen
    rec = coracle.rx_batch(buf[:end], n, stride=stride, frame_len=flen, nthreads=NTHREADS)
    res = lp.rx_process(to_dev(buf), stride=stride, frame_len=flen, n_frames=n, columns=ALL_COLUMNS,
                        data_bytes=end)
    torch.cuda.synchronize()
    compare(res, rec)
    assert (res.numpy()["status"] & 0x400).all()   # every L4 checksum verifies


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_stream_extension_dispatch(flags):
    rng = np.random.default_rng(60 + flags)
    frames = framegen.extension_frames(rng) + [
        framegen.add_vlan(framegen.build_frame(rng, k, 1400), [(0x8100, i), (0x88A8, i + 1)][: 1 + i % 2])
        for i, k in enumerate(("udp", "tcp", "icmp") * 40)]
    stride = 1536
    buf = stride_batch(rng, frames, stride, 6)
    rec = coracle.rx_batch(buf, len(frames), first=6, stride=stride, frame_len=stride, flags=flags,
                           nthreads=NTHREADS)
    res = lp.rx_process(to_dev(buf), stride=stride, frame_len=stride, first_offset=6, n_frames=len(frames),
                        columns=ALL_COLUMNS, flags=flags)
    torch.cuda.synchronize()
    compare(res, rec)


def test_stream_many_runs_per_wave():
    """More runs than waves in the grid: the ring prefetch crosses from one run
    into the next many times (2^17 frames of 1024 B, planted corruptions)."""
    rng = np.random.default_rng(5)
    n, stride = 1 << 17, 1024
    base = [framegen.build_frame(rng, k, stride - 34) for k in ("udp", "tcp")]
    buf = np.empty(n * stride + 64, np.uint8)
    for i in range(2):
        buf[i * stride:(i + 1) * stride] = np.frombuffer(base[i], np.uint8)
    buf[:n * stride].reshape(n, stride)[:] = buf[:2 * stride].reshape(2, stride)[np.arange(n) % 2]
    bad = rng.choice(n, 300, replace=False)
    pos = rng.integers(14, stride, 300)
    buf[bad * stride + pos] ^= 0x5A
    rec = coracle.rx_batch(buf, n, stride=stride, frame_len=stride, nthreads=NTHREADS)
    res = lp.rx_process(to_dev(buf), stride=stride, frame_len=stride, n_frames=n, columns=lp.IPV4_COLUMNS)
    torch.cuda.synchronize()
    compare(res, rec)
