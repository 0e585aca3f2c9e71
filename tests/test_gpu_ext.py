"""GPU parity of the opt-in dispatch extensions (PNETGPU_RX_VLAN,
PNETGPU_RX_IPV6_EXT) vs the oracle: descriptor mode at arbitrary alignment
(L4 headers beyond the LDS window included), fixed-stride mode, and TX fill."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import compare, to_dev

pytestmark = pytest.mark.gpu
FLAGS = [0, 1, 2, 3]


@pytest.mark.parametrize("flags", FLAGS)
def test_extension_frames_desc(flags):
    rng = np.random.default_rng(40 + flags)
    frames = framegen.extension_frames(rng) + framegen.random_frames(rng, 800)
    buf, offs, lens = framegen.pack(frames, gap=13, rng=rng)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    for data_offset in (0, 3):
        d = to_dev(np.concatenate([np.zeros(16, np.uint8), buf]))[data_offset:]
        res = lp.rx_process(d, offsets=to_dev((offs + 16 - data_offset).astype(np.int64)),
                            lengths=to_dev(lens.astype(np.int32)), columns=ALL_COLUMNS, flags=flags)
        torch.cuda.synchronize()
        compare(res, rec)


@pytest.mark.parametrize("flags", [1, 3])
def test_vlan_stride_mode(flags):
    rng = np.random.default_rng(7)
    frames = [framegen.add_vlan(framegen.build_frame(rng, "udp", 22), [(0x8100, i)]) for i in range(1000)]
    stride = 64
    buf = np.zeros(stride * len(frames) + 32, np.uint8)
    for i, f in enumerate(frames):
        buf[i * stride:i * stride + len(f)] = np.frombuffer(f, np.uint8)
    rec = coracle.rx_batch(buf, len(frames), stride=stride, frame_len=len(frames[0]), flags=flags)
    res = lp.rx_process(to_dev(buf), stride=stride, frame_len=len(frames[0]), n_frames=len(frames),
                        columns=ALL_COLUMNS, flags=flags)
    torch.cuda.synchronize()
    compare(res, rec)
    assert (res.numpy()["l3_offset"] == 18).all()


@pytest.mark.parametrize("flags", [3])
def test_tx_fill_with_extensions(flags):
    rng = np.random.default_rng(77)
    frames = framegen.extension_frames(rng)
    buf, offs, lens = framegen.pack(frames, gap=7, rng=rng)
    d = to_dev(buf.copy())
    res = lp.tx_fill_checksums(d, offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                               columns=ALL_COLUMNS, flags=flags)
    want_buf, want_rec = coracle.tx_fill(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), want_buf)
    compare(res, want_rec)


@pytest.mark.parametrize("flags", [4, 6, 7])
def test_l3_packets_desc(flags):
    """PNETGPU_RX_L3 (frames begin at the IP header) at arbitrary alignment."""
    from tests.test_oracle_ext import ip_packets
    rng = np.random.default_rng(50 + flags)
    pkts = ip_packets(rng, 1500)
    buf, offs, lens = framegen.pack(pkts, gap=11, rng=rng)
    rec = coracle.rx_batch(buf, len(pkts), offsets=offs, lengths=lens, flags=flags)
    for data_offset in (0, 5):
        d = to_dev(np.concatenate([np.zeros(16, np.uint8), buf]))[data_offset:]
        res = lp.rx_process(d, offsets=to_dev((offs + 16 - data_offset).astype(np.int64)),
                            lengths=to_dev(lens.astype(np.int32)), columns=ALL_COLUMNS, flags=flags)
        torch.cuda.synchronize()
        compare(res, rec)


def test_l3_stride_mode_and_tx_fill():
    """Fixed-stride L3 batches (raw IPv4/UDP datagrams of a sender) through the
    generic kernel, and the TX fill of their checksums in place."""
    rng = np.random.default_rng(9)
    pkts = [framegen.build_frame(rng, k, 30)[14:] for k in ("udp", "tcp", "icmp", "udp6", "tcp6") * 400]
    stride = 96
    buf = np.zeros(stride * len(pkts) + 32, np.uint8)
    for i, p in enumerate(pkts):
        buf[i * stride:i * stride + len(p)] = np.frombuffer(p, np.uint8)
    flen = max(len(p) for p in pkts)
    rec = coracle.rx_batch(buf, len(pkts), stride=stride, frame_len=flen, flags=4)
    res = lp.rx_process(to_dev(buf), stride=stride, frame_len=flen, n_frames=len(pkts), columns=ALL_COLUMNS, flags=4)
    torch.cuda.synchronize()
    compare(res, rec)
    st = res.numpy()["status"]
    assert ((st & 0x100) != 0).sum() == 1200 and ((st & 0x400) != 0).all()
    # zero every checksum field, fill them on the GPU: the original bytes come back
    z = buf.copy()
    for i in range(len(pkts)):
        r = rec[i]
        if r["status"] & 1:
            z[i * stride + 10:i * stride + 12] = 0
        if r["status"] & 0x200:
            at = int(r["l4_offset"]) + {4: 6, 8: 16, 12: 2, 16: 2}[int(r["status"]) & 0x1C]
            z[i * stride + at:i * stride + at + 2] = 0
    d = to_dev(z)
    lp.tx_fill_checksums(d, stride=stride, frame_len=flen, n_frames=len(pkts), flags=4)
    torch.cuda.synchronize()
    want, _ = coracle.tx_fill(z, len(pkts), stride=stride, frame_len=flen, flags=4)
    got = d.cpu().numpy()
    assert np.array_equal(got, want)
    assert np.array_equal(got, buf)


def _fuzz_batch(rng, n, max_len=1600):
    """n frames of random bytes, steered so most reach the IP and L4 parsers:
    ethertypes IPv4 / IPv6 / VLAN TPIDs / random, version nibbles 4 / 6,
    protocol and next-header bytes from the dispatch and extension sets."""
    lens = rng.integers(0, max_len, n).astype(np.uint32)
    short = rng.random(n) < 0.1                                # many frames around the minimum sizes
    lens[short] = rng.integers(0, 80, int(short.sum()))
    gaps = rng.integers(0, 24, n).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + gaps)[:-1]]).astype(np.uint64)
    buf = rng.integers(0, 256, int(offs[-1]) + int(lens[-1]) + 64, dtype=np.uint8)
    protos = np.array([6, 17, 1, 58, 0, 43, 44, 60, 47, 253], np.uint8)
    for i in np.nonzero(lens >= 14)[0]:
        o, ln = int(offs[i]), int(lens[i])
        r = rng.random()
        l3 = 14
        if r < 0.15:
            buf[o + 12:o + 14] = (0x81, 0x00)                   # one VLAN tag, then IP
            l3 = 18
            r = rng.random() * 0.8
        if l3 + 1 >= ln:
            continue
        if r < 0.45:
            buf[o + l3 - 2:o + l3] = (0x08, 0x00)
            buf[o + l3] = 0x40 | int(rng.integers(0, 16))
            if ln > l3 + 9:
                buf[o + l3 + 9] = protos[int(rng.integers(0, len(protos)))]
        elif r < 0.8:
            buf[o + l3 - 2:o + l3] = (0x86, 0xDD)
            buf[o + l3] = 0x60 | int(rng.integers(0, 16))
            if ln > l3 + 6:
                buf[o + l3 + 6] = protos[int(rng.integers(0, len(protos)))]
    return buf, offs, lens


@pytest.mark.parametrize("flags", [0, 3, 4, 7])
def test_fuzz_random_bytes_bit_exact(flags):
    """200k steered random frames per flag set, every column bit-exact vs the
    oracle (the reference's fuzz contract, fuzz/fuzzers/*.rs: arbitrary bytes
    parse without fault; here also without a single differing bit)."""
    rng = np.random.default_rng(1000 + flags)
    buf, offs, lens = _fuzz_batch(rng, 200_000)
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens, flags=flags, nthreads=16)
    res = lp.rx_process(to_dev(buf), offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                        columns=ALL_COLUMNS, flags=flags)
    torch.cuda.synchronize()
    compare(res, rec)


@pytest.mark.parametrize("flags", [0, 7])
def test_fuzz_tx_fill_bit_exact(flags):
    """TX fill over steered random bytes: the patched buffer (every checksum field
    the dispatch reaches, nothing else) equals the oracle's byte for byte."""
    rng = np.random.default_rng(2000 + flags)
    buf, offs, lens = _fuzz_batch(rng, 100_000)
    d = to_dev(buf.copy())
    res = lp.tx_fill_checksums(d, offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                               columns=ALL_COLUMNS, flags=flags)
    want_buf, want_rec = coracle.tx_fill(buf, len(offs), offsets=offs, lengths=lens, flags=flags)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    assert np.array_equal(got, want_buf), int((got != want_buf).sum())
    compare(res, want_rec)


@pytest.mark.parametrize("frame_len", [14, 20, 34, 42, 47, 60, 64])
def test_fuzz_small_kernel_bit_exact(frame_len):
    """rx_small_kernel (fixed 64-B stride) over steered random bytes: its register
    fast path and its fallback to the generic parse, bit-exact, TX fill too."""
    rng = np.random.default_rng(3000 + frame_len)
    n = 1 << 17
    buf = rng.integers(0, 256, n * 64 + 64, dtype=np.uint8)
    f = buf[: n * 64].reshape(n, 64)
    r = rng.random(n)
    f[r < 0.7, 12], f[r < 0.7, 13] = 0x08, 0x00
    f[(r >= 0.7) & (r < 0.85), 12], f[(r >= 0.7) & (r < 0.85), 13] = 0x86, 0xDD
    f[r < 0.7, 14] = 0x40 | rng.integers(0, 16, int((r < 0.7).sum())).astype(np.uint8)
    f[r < 0.5, 14] = 0x45                                          # mostly the fast path
    f[:, 23] = np.array([6, 17, 1, 58, 47], np.uint8)[rng.integers(0, 5, n)]
    short_tl = rng.random(n) < 0.3
    f[short_tl, 16] = 0
    f[short_tl, 17] = rng.integers(0, 64, int(short_tl.sum())).astype(np.uint8)
    rec = coracle.rx_batch(buf, n, stride=64, frame_len=frame_len, nthreads=16)
    res = lp.rx_process(to_dev(buf), stride=64, frame_len=frame_len, n_frames=n, columns=ALL_COLUMNS)
    torch.cuda.synchronize()
    compare(res, rec)
    d = to_dev(buf.copy())
    lp.tx_fill_checksums(d, stride=64, frame_len=frame_len, n_frames=n)
    want, _ = coracle.tx_fill(buf, n, stride=64, frame_len=frame_len)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), want)
