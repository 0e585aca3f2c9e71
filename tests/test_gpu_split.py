"""GPU parity of the split kernel (PNETGPU_RX_KIND=6: a streaming wave and two
parsing waves per block, receive only) against the oracle: packed and gapped
descriptor batches (compact and full, with and without the parse extensions),
shuffled / overlapping / empty / 65535-B frames (runs that are not packed take
the per-lane path), dense and spread runs interleaved, runs of minimum-size
frames (one ring step per run), fixed-stride batches, a batch ending at the
buffer's last byte, header-field columns, and the full-size BASELINE workloads
against the default kernels' records."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def split_kind(monkeypatch):
    monkeypatch.setenv("PNETGPU_RX_KIND", "6")


def rx(d, offs, lens, flags=0, compact=True, columns=ALL_COLUMNS):
    if compact:
        res = lp.rx_process(d, offsets=to_dev(np.asarray(offs, np.uint32).view(np.int32)),
                            lengths=to_dev(np.asarray(lens, np.uint16).view(np.int16)), columns=columns,
                            flags=flags | lp.DESC_COMPACT)
    else:
        res = lp.rx_process(d, offsets=to_dev(np.asarray(offs, np.uint64).view(np.int64)),
                            lengths=to_dev(np.asarray(lens, np.uint32).view(np.int32)), columns=columns, flags=flags)
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("flags", [0, 3])
@pytest.mark.parametrize("gap", [0, 13])
@pytest.mark.parametrize("compact", [True, False])
def test_packed_and_gapped_frames(flags, gap, compact):
    rng = np.random.default_rng(600 + flags + gap)
    frames = framegen.extension_frames(rng) + framegen.random_frames(rng, 4000, max_len=9100)
    buf, offs, lens = framegen.pack(frames, gap=gap, rng=rng)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens, flags=flags)
    for data_offset in (0, 5):
        d = to_dev(np.concatenate([np.zeros(16, np.uint8), buf]))[data_offset:]
        res = rx(d, offs + 16 - data_offset, lens, flags=flags, compact=compact)
        compare(res, rec)
        assert res.counter_dict() == oracle_counters(rec, lens)


def test_any_order_overlaps_empty_and_max_length():
    rng = np.random.default_rng(604)
    frames = framegen.random_frames(rng, 3000, max_len=3000) + framegen.edge_frames(rng)
    buf, offs, lens = framegen.pack(frames, gap=7, rng=rng)
    offs, lens = offs.astype(np.uint64), lens.astype(np.uint32)
    big = rng.integers(0, 256, 70000, dtype=np.uint8)
    big[12:14] = (8, 0)
    big[14] = 0x45
    base = buf.size
    buf = np.concatenate([buf, big, np.zeros(32, np.uint8)])
    extra_o = [base + a for a in (0, 1, 7, 15, 16, 4000)] + [int(o) + 3 for o in offs[:200:7]] + [5, 9, base]
    extra_l = [65535, 65535, 65535, 65535, 60000, 65535 - 4000] + [max(0, int(n) - 5) for n in lens[:200:7]] + [0, 0, 0]
    offs = np.concatenate([offs, np.array(extra_o, np.uint64)])
    lens = np.concatenate([lens, np.array(extra_l, np.uint32)])
    perm = rng.permutation(len(offs))
    offs, lens = offs[perm], lens[perm]
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
    res = rx(to_dev(buf), offs, lens)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


def test_dense_and_spread_runs_interleaved():
    """Every other run of 64 frames shuffled across the whole buffer (not
    packed: the per-lane path), the others packed in place (streamed), and a
    run of overlapping copies of one frame (packed: its span is one frame)."""
    rng = np.random.default_rng(605)
    frames = framegen.random_frames(rng, 64 * 40, max_len=1600)
    buf, offs, lens = framegen.pack(frames, gap=0, rng=rng)
    offs, lens = offs.astype(np.uint64).copy(), lens.astype(np.uint32).copy()
    for r in range(1, 40, 2):
        sl = slice(64 * r, 64 * r + 64)
        p = rng.permutation(len(offs))[:64]
        offs[sl], lens[sl] = offs[p], lens[p]
    offs[64 * 6:64 * 7], lens[64 * 6:64 * 7] = offs[10], lens[10]
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
    for compact in (True, False):
        res = rx(to_dev(buf), offs, lens, compact=compact)
        compare(res, rec)
        assert res.counter_dict() == oracle_counters(rec, lens)


def test_minimum_size_frames_one_step_per_run():
    """Runs of 60-64-B frames: 4 KiB per run, so the ring's S-1 steps in flight
    span only the current and the next run."""
    rng = np.random.default_rng(606)
    frames = [framegen.build_frame(rng, "udp", int(rng.integers(18, 23))) for _ in range(64 * 300 + 17)]
    buf, offs, lens = framegen.pack(frames, gap=0, rng=rng)
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
    res = rx(to_dev(buf), offs, lens)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


def test_batch_ends_at_the_buffer_end():
    """The last frame's last byte is the buffer's last byte (the ring's last
    step re-reads the buffer's last granule past it), at every end alignment."""
    rng = np.random.default_rng(607)
    for tail in range(16):
        frames = framegen.random_frames(rng, 700, max_len=1600)
        buf, offs, lens = framegen.pack(frames, gap=0, rng=rng)
        buf = buf[:int(offs[-1] + lens[-1])]
        extra = np.zeros(tail, np.uint8)
        buf = np.concatenate([extra, buf])
        offs = offs + tail
        rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens)
        res = rx(to_dev(buf), offs, lens)
        compare(res, rec)


@pytest.mark.parametrize("stride,flen", [(150, 97), (1500, 1500), (1514, 1400), (9018, 9000)])
def test_fixed_stride(stride, flen):
    rng = np.random.default_rng(608 + stride)
    n = 64 * 37 + 5
    frames = [framegen.build_frame(rng, rng.choice(["udp", "tcp", "icmp"]), flen - 42) for _ in range(n)]
    buf = np.zeros(n * stride + 3, np.uint8)
    for i, f in enumerate(frames):
        f = np.frombuffer(bytes(f)[:flen], np.uint8)
        buf[3 + i * stride:3 + i * stride + f.size] = f
    offs = np.arange(n, dtype=np.uint64) * stride + 3
    lens = np.full(n, flen, np.uint32)
    rec = coracle.rx_batch(buf, n, offsets=offs, lengths=lens)
    res = lp.rx_process(to_dev(buf), stride=stride, frame_len=flen, n_frames=n, first_offset=3, columns=ALL_COLUMNS)
    torch.cuda.synchronize()
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


@pytest.mark.parametrize("name", ["imix", "tcp1500", "udp6_jumbo"])
def test_workloads_full_size_equal_default_kernels(name, monkeypatch):
    n = {"imix": 1 << 22, "tcp1500": 1 << 20, "udp6_jumbo": 1 << 17}[name]
    w = lp.synth.make(name, n, seed=11, corrupt_ppm=10000)
    d = to_dev(w.buf)

    def run():
        if w.stride:
            r = lp.rx_process(d, stride=w.stride, frame_len=w.frame_len, n_frames=n, columns=lp.IPV4_COLUMNS
                              if name != "udp6_jumbo" else ALL_COLUMNS)
        else:
            r = rx(d, w.offsets, w.lengths, columns=lp.IPV4_COLUMNS)
        torch.cuda.synchronize()
        return r

    got = run()
    monkeypatch.delenv("PNETGPU_RX_KIND")
    want = run()
    a, b = got.numpy(), want.numpy()
    for c in a:
        assert np.array_equal(a[c], b[c]), c
    assert got.counter_dict() == want.counter_dict()
    assert got.counter_dict()["frames"] == n


def test_header_field_columns():
    """The EXT instantiation with every header-field column, on packed frames."""
    rng = np.random.default_rng(609)
    frames = framegen.extension_frames(rng) + framegen.random_frames(rng, 3000, max_len=2000)
    buf, offs, lens = framegen.pack(frames, gap=0, rng=rng)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens)
    res = rx(to_dev(buf), offs, lens, columns=ALL_COLUMNS)
    compare(res, rec)


@pytest.mark.parametrize("per_cu", ["1", "2"])
def test_many_runs_per_block(per_cu, monkeypatch):
    """Few blocks (PNETGPU_BLOCKS_PER_CU) so every block takes several runs —
    odd and even counts, the pair schedule's last period with one run — with
    every fifth run spread out (per-lane path) between streamed ones."""
    monkeypatch.setenv("PNETGPU_BLOCKS_PER_CU", per_cu)
    rng = np.random.default_rng(610)
    n = 64 * 1000 + 33
    frames = framegen.random_frames(rng, n, max_len=600)
    buf, offs, lens = framegen.pack(frames, gap=0, rng=rng)
    offs, lens = offs.astype(np.uint64).copy(), lens.astype(np.uint32).copy()
    for r in range(3, n // 64, 5):
        sl = slice(64 * r, 64 * r + 64)
        p = rng.permutation(n)[:64]
        offs[sl], lens[sl] = offs[p], lens[p]
    rec = coracle.rx_batch(buf, n, offsets=offs, lengths=lens)
    res = rx(to_dev(buf), offs, lens)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


@pytest.mark.parametrize("flags", [4, 7])
def test_l3_packets(flags):
    """PNETGPU_RX_L3 batches (frames begin at the IP header), with and without
    the other extensions, packed (streamed) at an odd base."""
    from tests.test_oracle_ext import ip_packets
    rng = np.random.default_rng(611 + flags)
    pkts = ip_packets(rng, 3000)
    buf, offs, lens = framegen.pack(pkts, gap=0, rng=rng)
    rec = coracle.rx_batch(buf, len(pkts), offsets=offs, lengths=lens, flags=flags)
    d = to_dev(np.concatenate([np.zeros(16, np.uint8), buf]))[3:]
    res = rx(d, offs + 13, lens, flags=flags)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)
