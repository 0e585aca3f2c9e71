"""GPU parity of the sender side (pnetgpu_tx_fill_checksums) vs oracle_tx_fill:
the patched frame buffer is byte-identical and the (pre-patch) records match,
through both kernels (small fixed-stride and generic descriptor mode)."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS
from oracle import coracle, pyoracle
from tests import framegen
from tests.test_gpu_parity import compare, to_dev

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,n", [("udp64", 1 << 18), ("tcp1500", 1 << 14), ("imix", 1 << 16),
                                    ("udp6_jumbo", 1 << 10)])
def test_tx_fill_workloads(name, n):
    w = lp.synth.make(name, n, seed=12, corrupt_ppm=300000)
    d = to_dev(w.buf.copy())
    if w.stride:
        res = lp.tx_fill_checksums(d, stride=w.stride, frame_len=w.frame_len, n_frames=n, columns=ALL_COLUMNS)
        want_buf, want_rec = coracle.tx_fill(w.buf, n, stride=w.stride, frame_len=w.frame_len)
    else:
        res = lp.tx_fill_checksums(d, offsets=to_dev(w.offsets.astype(np.int64)),
                                   lengths=to_dev(w.lengths.astype(np.int32)), columns=ALL_COLUMNS)
        want_buf, want_rec = coracle.tx_fill(w.buf, n, offsets=w.offsets, lengths=w.lengths)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    assert np.array_equal(got, want_buf), f"{int((got != want_buf).sum())} bytes differ"
    compare(res, want_rec)


def test_tx_fill_edge_and_random_frames_any_alignment():
    rng = np.random.default_rng(31)
    frames = framegen.edge_frames(rng) + framegen.random_frames(rng, 3000, max_len=3000)
    buf, offs, lens = framegen.pack(frames, gap=9, rng=rng)
    d = to_dev(buf.copy())
    res = lp.tx_fill_checksums(d, offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                               columns=ALL_COLUMNS)
    want_buf, want_rec = coracle.tx_fill(buf, len(frames), offsets=offs, lengths=lens)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), want_buf)
    compare(res, want_rec)


def test_tx_then_rx_all_verify_and_idempotent():
    w = lp.synth.make("udp64", 1 << 16, seed=2, corrupt_ppm=500000)
    d = to_dev(w.buf.copy())
    lp.tx_fill_checksums(d, stride=64, frame_len=64, n_frames=w.n)
    once = d.clone()
    lp.tx_fill_checksums(d, stride=64, frame_len=64, n_frames=w.n)
    assert torch.equal(d, once)
    r = lp.rx_process(d, stride=64, frame_len=64, n_frames=w.n)
    c = r.counter_dict()
    assert c["ip_csum_bad"] == 0 and c["l4_csum_bad"] == 0 and c["frames"] == w.n


@pytest.mark.parametrize("stride,flen", [(64, 64), (64, 60), (1514, 1514), (1500, 1400), (9018, 9018)])
def test_tx_fill_stride_every_kernel(stride, flen, tune):
    """Fixed-stride TX fill of random/corrupted frames through the default kernel
    for the shape and every forced rx_kernel kind (the rx_kind tuning)."""
    rng = np.random.default_rng(stride * 7 + flen)
    n = 300
    frames = framegen.random_frames(rng, n, max_len=min(stride, 9100))
    buf = rng.integers(0, 256, stride * n + 64, dtype=np.uint8)
    for i, f in enumerate(frames):
        f = np.frombuffer(f, np.uint8)[:stride]
        buf[i * stride:i * stride + len(f)] = f
    want_buf, want_rec = coracle.tx_fill(buf, n, stride=stride, frame_len=flen)
    for kind in (None, "0", "2", "3"):
        tune("rx_kind", None if kind is None else int(kind))
        d = to_dev(buf.copy())
        res = lp.tx_fill_checksums(d, stride=stride, frame_len=flen, n_frames=n, columns=ALL_COLUMNS)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        assert np.array_equal(got, want_buf), (kind, int((got != want_buf).sum()))
        compare(res, want_rec)


def test_payload_mut_then_gpu_fill():
    """MutablePacket::payload_mut on host frame buffers (libpnet_amd.views), the
    payloads edited, then tx_fill_checksums on the GPU: the frames equal the
    oracle's fill of the same edited bytes and verify on the receive path."""
    rng = np.random.default_rng(23)
    frames = [framegen.build_frame(rng, k, 40 + 3 * i) for i, k in enumerate(("udp", "tcp", "icmp", "udp6", "tcp6") * 20)]
    buf, offs, lens = framegen.pack(frames, gap=3, rng=rng)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens)
    edit = buf.copy()
    for i in range(len(frames)):
        fr = edit[int(offs[i]):int(offs[i]) + int(lens[i])]          # a writable numpy view into the batch
        v = lp.frame_view(rec, i, fr)
        ip = v.ipv4() or v.ipv6()
        l4 = ip.udp() or ip.tcp() or ip.icmp()
        pm = l4.payload_mut()
        pm[:4] = bytes([i & 0xFF, 0x55, 0xAA, 0x01])
    assert not np.array_equal(edit, buf)
    d = to_dev(edit)
    lp.tx_fill_checksums(d, offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)))
    torch.cuda.synchronize()
    want_buf, _ = coracle.tx_fill(edit, len(frames), offsets=offs, lengths=lens)
    got = d.cpu().numpy()
    assert np.array_equal(got, want_buf)
    after = coracle.rx_batch(got, len(frames), offsets=offs, lengths=lens)
    assert ((after["status"] & 0x0400) != 0).all()
