"""GPU parity: libpnetgpu.so (HIP, through the C-ABI) vs the CPU oracle.

Bit-exact on every column for: the reference's own KAT vectors, the edge-case
set, random/malformed frames at arbitrary byte alignment, every BASELINE
workload at full per-GPU size (BASELINE.json configs 2-5), and the batched
util::checksum / ipv4_checksum / ipv6_checksum entry points.
"""
import os
import re

import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS, COLUMNS, RECORD_COLUMNS
from oracle import coracle, pyoracle
from tests import framegen, kats

pytestmark = pytest.mark.gpu
NTHREADS = min(16, os.cpu_count() or 1)
DEV = "cuda:0"


# rx_kernel's tail shapes by template arguments <NW, G, U, NT, PASS, DYN, ...>
# (the window granules NW may differ per build: regex)
SHAPE_RE = {"mixed": r"rx_kernel<\d+, 4, 8, false, 0, true, ", "mtu": r"rx_kernel<\d+, 8, 4, false, 1, false, ",
            "jumbo": r"rx_kernel<\d+, 64, 9, true, 0, false, "}


def to_dev(a, dtype=None):
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:
        a = a.copy()
    t = torch.from_numpy(a)
    if dtype is not None:
        t = t.view(dtype)
    return t.to(DEV)


def compare(res, rec, idx=None):
    """Every column of an RxResult equals the oracle records."""
    got = res.numpy()
    for c in res.columns:
        exp = rec[c]
        g = got[c]
        if idx is not None:
            g = g[idx]
        if not np.array_equal(g, exp):
            bad = np.nonzero((g != exp).reshape(len(exp), -1).any(axis=1))[0]
            i = int(bad[0])
            raise AssertionError(f"column {c}: {len(bad)} mismatches, first at {i}: got {g[i]} want {exp[i]} "
                                 f"(status want {rec['status'][i]:#x})")


def run_desc(buf, offs, lens, columns=ALL_COLUMNS, data_offset=0):
    d = to_dev(buf)
    if data_offset:
        d = d[data_offset:]
        offs = offs - data_offset
    res = lp.rx_process(d, offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                        columns=columns)
    torch.cuda.synchronize()
    return res


def oracle_desc(buf, offs, lens):
    return coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens, nthreads=NTHREADS)


def oracle_counters(rec, lens):
    st = rec["status"].astype(np.int64)
    valid = (st & pyoracle.ST_DESC_INVALID) == 0
    return {
        "frames": int(valid.sum()),
        "bytes": int(lens[valid].astype(np.int64).sum()),
        "ipv4": int(((st & 3) == 1).sum()),
        "ipv6": int(((st & 3) == 2).sum()),
        "ip_csum_bad": int((((st & 3) == 1) & ((st & 0x40) == 0) & ((st & 0x100) == 0)).sum()),
        "l4_csum_bad": int((((st & 0x200) != 0) & ((st & 0x400) == 0)).sum()),
        "malformed": int(((st & (0x20 | 0x40 | 0x80 | 0x8000)) != 0).sum()),
        "unknown": int(((st & (0x800 | 0x1000)) != 0).sum()),
    }


# ---- reference KATs -------------------------------------------------------

def test_kat_checksum_slices():
    vs = kats.by_kind("sum_be_words", "checksum")
    for misalign in (0, 1, 2, 3, 5, 15):
        parts, offs, lens, skips, want = [], [], [], [], []
        pos = 0
        for v in vs:
            pad = (misalign - pos) % 16
            parts.append(bytes(pad))
            pos += pad
            offs.append(pos)
            lens.append(len(v["data"]))
            skips.append(v["skipword"])
            parts.append(v["data"])
            pos += len(v["data"])
            if v["kind"] == "checksum":
                want.append(v["expected"])
            else:  # sum_be_words: util::checksum = finalize(sum) for non-empty data
                want.append(pyoracle.finalize(v["expected"]) if v["data"] else 0)
        buf = np.frombuffer(b"".join(parts) + bytes(32), dtype=np.uint8)
        out = lp.checksum_slices(to_dev(buf), to_dev(np.array(offs, np.int64)), to_dev(np.array(lens, np.int32)),
                                 to_dev(np.array(skips, np.int32)))
        got = out.cpu().numpy().view(np.uint16)
        assert list(got) == want, misalign


def test_kat_pseudo_header_slices():
    for kind, fn, alen in (("ipv4_checksum", lp.ipv4_checksum_slices, 8),
                           ("ipv6_checksum", lp.ipv6_checksum_slices, 32)):
        vs = kats.by_kind(kind)
        buf = b""
        offs, lens, skips, addrs, protos = [], [], [], [], []
        for k, v in enumerate(vs):
            buf += bytes(k % 7)
            offs.append(len(buf))
            lens.append(len(v["data"]))
            buf += v["data"]
            skips.append(v["skipword"])
            addrs.append(bytes(v["src"]) + bytes(v["dst"]))
            protos.append(v["proto"])
        b = np.frombuffer(buf + bytes(32), dtype=np.uint8)
        out = fn(to_dev(b), to_dev(np.array(offs, np.int64)), to_dev(np.array(lens, np.int32)),
                 to_dev(np.array(skips, np.int32)), to_dev(np.frombuffer(b"".join(addrs), np.uint8).reshape(-1, alen)),
                 to_dev(np.array(protos, np.uint8)))
        assert list(out.cpu().numpy().view(np.uint16)) == [v["expected"] for v in vs], kind


def test_kat_frames_rx():
    frames, expect = [], []
    for v in kats.by_kind("ipv4_header"):
        frames.append(bytes(12) + b"\x08\x00" + v["data"])
        expect.append(("ip_csum", v["expected"]))
    for v in kats.by_kind("rx_frame"):
        frames.append(v["data"])
        expect.append(("l4_csum", v["expected"]["l4_csum"]))
    buf, offs, lens = framegen.pack(frames)
    res = run_desc(buf, offs, lens)
    got = res.numpy()
    for i, (col, val) in enumerate(expect):
        assert got[col][i] == val, (i, col)
    compare(res, oracle_desc(buf, offs, lens))


def test_kat_header_getters():
    """The header-field columns (ABI v3) hold the values the reference's own tests
    assert for ethernet.rs / ipv4.rs / ipv6.rs / udp.rs / tcp.rs getters, through
    the descriptor kernel at several alignments, and every column equals the oracle."""
    vs = kats.by_kind("getters")
    frames = [kats.getter_frame(v) for v in vs]
    for gap in (0, 5):
        buf, offs, lens = framegen.pack(frames, gap=gap, rng=np.random.default_rng(gap))
        res = run_desc(buf, offs, lens)
        got = res.numpy()
        for i, v in enumerate(vs):
            for k, want in v["expected"].items():
                assert int(got[k][i]) == want, (v["name"], k)
        compare(res, oracle_desc(buf, offs, lens))


def test_icmp_sequence_echo_types_only():
    """icmp_sequence on the GPU: the echo views' sequence number for ICMP 0/8 and
    ICMPv6 128/129 with >= 8 B, 0 for every other type, at two alignments."""
    frames, echo = framegen.icmp_type_frames(np.random.default_rng(9))
    for gap in (0, 3):
        buf, offs, lens = framegen.pack(frames, gap=gap, rng=np.random.default_rng(gap))
        res = run_desc(buf, offs, lens)
        got = res.numpy()
        for i, e in enumerate(echo):
            if not e:
                assert got["icmp_sequence"][i] == 0, i
        compare(res, oracle_desc(buf, offs, lens))


# ---- edge cases, random frames, alignment ---------------------------------

@pytest.mark.parametrize("gap", [0, 3, 15])
def test_edge_frames(gap):
    rng = np.random.default_rng(11)
    frames = framegen.edge_frames(rng)
    buf, offs, lens = framegen.pack(frames, gap=gap, rng=rng)
    res = run_desc(buf, offs, lens)
    rec = oracle_desc(buf, offs, lens)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


@pytest.mark.parametrize("seed", [0, 1])
def test_random_frames_any_alignment(seed):
    rng = np.random.default_rng(100 + seed)
    frames = framegen.random_frames(rng, 6000, max_len=9100)
    buf, offs, lens = framegen.pack(frames, gap=17, rng=rng)
    rec = oracle_desc(buf, offs, lens)
    for data_offset in (0, 1, 6):
        res = run_desc(np.concatenate([np.zeros(64, np.uint8), buf]), offs + 64, lens, data_offset=data_offset)
        compare(res, rec)


def test_invalid_descriptors_and_partial_columns():
    rng = np.random.default_rng(5)
    frames = framegen.random_frames(rng, 500)
    buf, offs, lens = framegen.pack(frames)
    offs = offs.copy()
    lens = lens.copy()
    offs[3] = buf.size + 100
    lens[7] = buf.size
    offs[11] = (1 << 40) + 7   # wild and misaligned: must be flagged, never dereferenced
    rec = oracle_desc(buf, offs, lens)
    assert rec["status"][3] == pyoracle.ST_DESC_INVALID == rec["status"][7] == rec["status"][11]
    res = run_desc(buf, offs, lens, columns=("status", "l4_csum", "src_ipv6"))
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


def test_descriptors_at_the_buffer_end():
    """Descriptors ending exactly at, one byte past, and far past the end of the
    buffer, at every alignment: in-bounds ones parse, the others are flagged
    DESC_INVALID (nothing is read for them), every column equal to the oracle."""
    rng = np.random.default_rng(17)
    frames = framegen.random_frames(rng, 300)
    buf, offs, lens = framegen.pack(frames)
    size = buf.size
    offs = offs.astype(np.uint64).copy()
    lens = lens.astype(np.uint32).copy()
    k = 0
    for sh in range(16):                                  # ends exactly at the buffer end
        lens[k] = 20 + sh
        offs[k] = size - lens[k]
        k += 1
    for sh in range(16):                                  # one byte past the end
        lens[k] = 40 + sh
        offs[k] = size - lens[k] + 1
        k += 1
    for v in (size, size + 1, size + 15, 2**32 + 3, 2**48 + 9, 2**63 + 5):   # start at / past the end
        offs[k] = v
        lens[k] = 64
        k += 1
    offs[k] = 0                                           # length past the end, and a length overflowing off+len
    lens[k] = size + 1
    offs[k + 1] = 5
    lens[k + 1] = 2**32 - 1
    rec = oracle_desc(buf, offs, lens)
    st = rec["status"]
    assert not (st[:16] & pyoracle.ST_DESC_INVALID).any()
    assert (st[16:k + 2] & pyoracle.ST_DESC_INVALID).all()
    res = run_desc(buf, offs.view(np.int64), lens.view(np.int32))
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)


def test_stride_mode_odd_stride_and_offset():
    rng = np.random.default_rng(8)
    frames = [framegen.build_frame(rng, k, 77) for k in ("udp", "tcp", "icmp", "udp6", "tcp6", "icmp6")] * 50
    stride = 150
    buf = np.zeros(7 + stride * len(frames) + 32, np.uint8)
    for i, f in enumerate(frames):
        buf[7 + i * stride:7 + i * stride + len(f)] = np.frombuffer(f, np.uint8)
    for flen in (stride, 91, 13):
        rec = coracle.rx_batch(buf, len(frames), first=7, stride=stride, frame_len=flen)
        res = lp.rx_process(to_dev(buf), stride=stride, frame_len=flen, first_offset=7, n_frames=len(frames),
                            columns=ALL_COLUMNS)
        torch.cuda.synchronize()
        compare(res, rec)


@pytest.mark.parametrize("stride", [16, 48, 64, 80, 128])
def test_small_kernel_strides_and_lengths(stride):
    """The register-resident small kernel (fixed stride, multiple of 16, frames
    <= 64 B, 16-B aligned): every frame length from the Ethernet minimum edge to
    64 B, random kinds (IPv6 and IPv4 options take its generic slow path),
    corrupted bytes, a batch that is not a whole number of 64-frame runs, and
    garbage between frames."""
    rng = np.random.default_rng(stride)
    n = 1000
    kinds = ("udp", "tcp", "icmp", "udp6", "tcp6", "icmp6", "icmp_over6")
    frames = []
    for i in range(n):
        k = kinds[i % len(kinds)]
        ihl = 5 if i % 5 else int(rng.integers(5, 16))
        f = bytearray(framegen.build_frame(rng, k, int(rng.integers(0, 40)), ihl=ihl))
        if i % 9 == 0 and len(f) > 20:
            f[int(rng.integers(14, len(f)))] ^= 0x5A
        frames.append(bytes(f))
    for first in (0, 32):
        for flen in sorted({0, 1, 13, 14, 33, 34, 41, 42, 53, 54, 61, 64, min(stride, 64)}):
            if flen > stride:
                continue
            buf = rng.integers(0, 256, first + stride * n + 64, dtype=np.uint8)
            for i, f in enumerate(frames):
                f = np.frombuffer(f, np.uint8)[:stride]
                buf[first + i * stride:first + i * stride + len(f)] = f
            rec = coracle.rx_batch(buf, n, first=first, stride=stride, frame_len=flen, nthreads=NTHREADS)
            res = lp.rx_process(to_dev(buf), stride=stride, frame_len=flen, first_offset=first, n_frames=n,
                                columns=ALL_COLUMNS)
            torch.cuda.synchronize()
            compare(res, rec)
            assert res.counter_dict() == oracle_counters(rec, np.full(n, flen, np.uint32)), (first, flen)


@pytest.mark.parametrize("stride,flen", [(144, 144), (150, 97), (333, 333), (1500, 1500), (1514, 1400),
                                         (4000, 3999), (9018, 9018)])
def test_stride_mode_random_frames_every_kernel(stride, flen, tune):
    """Fixed-stride batches of random/malformed frames (garbage between frames,
    L4 ranges shorter than the frame, IPv4 options, IPv6) at every first-offset
    alignment: the default kernel for the stride (rx_kernel's MTU shape below
    4 KiB, the jumbo shape from 4 KiB) and every rx_kernel shape forced through
    the rx_kind tuning (mixed, MTU, jumbo) all bit-exact."""
    rng = np.random.default_rng(stride + flen)
    n = 700
    frames = framegen.random_frames(rng, n, max_len=min(stride + 64, 9100))
    for first in (0, 5, 12):
        buf = rng.integers(0, 256, first + stride * n + 64, dtype=np.uint8)
        for i, f in enumerate(frames):
            f = np.frombuffer(f, np.uint8)[:stride]
            buf[first + i * stride:first + i * stride + len(f)] = f
        rec = coracle.rx_batch(buf, n, first=first, stride=stride, frame_len=flen, nthreads=NTHREADS)
        d = to_dev(buf)
        for kind in (None, "0", "2", "3"):
            tune("rx_kind", None if kind is None else int(kind))
            res = lp.rx_process(d, stride=stride, frame_len=flen, first_offset=first, n_frames=n,
                                columns=ALL_COLUMNS)
            torch.cuda.synchronize()
            compare(res, rec)
            lens = np.full(n, flen, np.uint32)
            assert res.counter_dict() == oracle_counters(rec, lens), (first, kind)


# ---- BASELINE workloads at full per-GPU size -------------------------------

FULL = {"udp64": 1 << 24, "tcp1500": 1 << 20, "udp1500": 1 << 20, "imix": 1 << 22, "udp6_jumbo": 1 << 17}


@pytest.mark.parametrize("name", list(FULL))
def test_workload_full_size_bit_exact(name):
    n = FULL[name]
    w = lp.synth.make(name, n, seed=3, corrupt_ppm=10000)
    d = to_dev(w.buf)
    cols = ALL_COLUMNS if name == "udp6_jumbo" else lp.IPV4_COLUMNS
    if w.stride:
        res = lp.rx_process(d, stride=w.stride, frame_len=w.frame_len, n_frames=n, columns=cols)
        rec = coracle.rx_batch(w.buf, n, stride=w.stride, frame_len=w.frame_len, nthreads=NTHREADS)
        lens = np.full(n, w.frame_len, np.uint32)
    else:
        res = lp.rx_process(d, offsets=to_dev(w.offsets.astype(np.int64)), lengths=to_dev(w.lengths.astype(np.int32)),
                            columns=cols)
        rec = coracle.rx_batch(w.buf, n, offsets=w.offsets, lengths=w.lengths, nthreads=NTHREADS)
        lens = w.lengths
    torch.cuda.synchronize()
    compare(res, rec)
    c = res.counter_dict()
    assert c == oracle_counters(rec, lens)
    # size-independent property: every planted corruption is detected, nothing else
    assert c["ip_csum_bad"] == w.expect["ip_bad"] and c["l4_csum_bad"] == w.expect["l4_bad"]
    assert c["bytes"] == w.expect["bytes"] and c["frames"] == n


@pytest.mark.parametrize("name", list(FULL))
def test_workload_full_size_header_fields(name):
    """Every header-field column at full per-GPU size, bit-exact with the oracle
    (udp64 exercises the small kernel's register path, tcp1500 the MTU kernel,
    imix the mixed kernel with UDP/TCP/ICMP echo, udp6_jumbo the IPv6 view)."""
    n = FULL[name]
    w = lp.synth.make(name, n, seed=5, corrupt_ppm=10000)
    d = to_dev(w.buf)
    cols = ("status",) + lp.FIELD_COLUMNS
    if w.stride:
        res = lp.rx_process(d, stride=w.stride, frame_len=w.frame_len, n_frames=n, columns=cols)
        rec = coracle.rx_batch(w.buf, n, stride=w.stride, frame_len=w.frame_len, nthreads=NTHREADS)
    else:
        res = lp.rx_process(d, offsets=to_dev(w.offsets.astype(np.int64)), lengths=to_dev(w.lengths.astype(np.int32)),
                            columns=cols)
        rec = coracle.rx_batch(w.buf, n, offsets=w.offsets, lengths=w.lengths, nthreads=NTHREADS)
    torch.cuda.synchronize()
    compare(res, rec)
    got = res.numpy()
    # the workload's views are really reached (not a trivially all-zero column)
    assert got["eth_dst"].any() or got["eth_src"].any()
    assert (got["ip_version"] != 0).mean() > 0.98


def test_descriptor_tensor_validation():
    """rx_process refuses descriptors the kernel would misread (host memory,
    another layout, strided views, more frames than descriptors) before any launch."""
    w = lp.synth.make("imix", 1000, seed=2)
    d = to_dev(w.buf)
    o, ln = to_dev(w.offsets.astype(np.int64)), to_dev(w.lengths.astype(np.int32))
    with pytest.raises(TypeError):
        lp.rx_process(d, offsets=o, lengths=ln.cpu())
    with pytest.raises(TypeError):
        lp.rx_process(d, offsets=o.cpu(), lengths=ln)
    with pytest.raises(TypeError):
        lp.rx_process(d, offsets=o[::2], lengths=ln[::2])
    with pytest.raises(TypeError):
        lp.rx_process(d, offsets=o.int(), lengths=ln)
    with pytest.raises(ValueError):
        lp.rx_process(d, offsets=o, lengths=ln, n_frames=1001)
    with pytest.raises(ValueError):
        lp.rx_process(d, offsets=o, lengths=ln[:500])
    with pytest.raises(TypeError):
        lp.rx_process(d, offsets=o, lengths=ln, flags=lp.DESC_COMPACT)
    small = lp.RxResult(10, DEV)
    with pytest.raises(ValueError):
        lp.rx_process(d, offsets=o, lengths=ln, out=small)
    res = lp.rx_process(d, offsets=o, lengths=ln, n_frames=600)   # a prefix of the descriptors is fine
    torch.cuda.synchronize()
    assert res.counter_dict()["frames"] == 600


def test_idempotent_and_stream_ordered():
    w = lp.synth.make("imix", 1 << 16, seed=4)
    d = to_dev(w.buf)
    o, l = to_dev(w.offsets.astype(np.int64)), to_dev(w.lengths.astype(np.int32))
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        a = lp.rx_process(d, offsets=o, lengths=l, stream=s)
        b = lp.rx_process(d, offsets=o, lengths=l, stream=s)
    s.synchronize()
    for c in a.columns:
        assert torch.equal(a.columns[c], b.columns[c])


@pytest.mark.parametrize("kernel", ["run", "group", "tiny"])
def test_random_slices_vs_oracle(kernel, tune):
    tune("slice_kernel", kernel)   # slice_run_kernel / slice_kernel / slice_tiny_kernel (util::checksum)
    rng = np.random.default_rng(21)
    n = 20000
    buf = rng.integers(0, 256, 1 << 22, dtype=np.uint8)
    lens = rng.integers(0, 3000, n).astype(np.uint32)
    offs = rng.integers(0, buf.size - 3100, n).astype(np.uint64)
    skips = rng.integers(0, 1600, n).astype(np.uint32)
    want = coracle.checksum_slices(buf, offs, lens, skips)
    got = lp.checksum_slices(to_dev(buf), to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)),
                             to_dev(skips.astype(np.int32)))
    assert np.array_equal(got.cpu().numpy().view(np.uint16), want)
    addrs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    protos = rng.integers(0, 256, n, dtype=np.uint8)
    for fn, alen, ofn in ((lp.ipv4_checksum_slices, 8, coracle.ipv4_checksum),
                          (lp.ipv6_checksum_slices, 32, coracle.ipv6_checksum)):
        a = np.ascontiguousarray(addrs[:, :alen])
        got = fn(to_dev(buf), to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)),
                 to_dev(skips.astype(np.int32)), to_dev(a), to_dev(protos)).cpu().numpy().view(np.uint16)
        for i in range(0, n, 97):
            o, ln = int(offs[i]), int(lens[i])
            h = alen // 2
            assert got[i] == ofn(bytes(buf[o:o + ln]), int(skips[i]), b"", bytes(a[i, :h]), bytes(a[i, h:]),
                                 int(protos[i])), i


@pytest.mark.parametrize("kernel", ["run", "group", "tiny"])
@pytest.mark.parametrize("seed", [0, 1])
def test_small_and_large_slices_mixed_in_runs(seed, kernel, tune):
    """slice_run_kernel: tiny slices (0-70 B, summed by their own lane) and long
    ones (group path) interleaved in the same 64-slice runs, at every alignment,
    skipwords inside / straddling / past the slice, invalid descriptors, and a
    batch size that is not a multiple of 64; pseudo-header forms with the
    address array at a 4-B-aligned and an odd address. Both slice kernels."""
    tune("slice_kernel", kernel)
    rng = np.random.default_rng(600 + seed)
    n = 64 * 300 + 17
    buf = rng.integers(0, 256, 1 << 21, dtype=np.uint8)
    lens = rng.integers(0, 71, n).astype(np.uint32)
    big = rng.random(n) < 0.2
    lens[big] = rng.integers(71, 5000, int(big.sum()))
    offs = rng.integers(0, buf.size - 5100, n).astype(np.uint64)
    skips = np.where(rng.random(n) < 0.5, rng.integers(0, 40, n), rng.integers(0, 3000, n)).astype(np.uint32)
    bad = rng.choice(n, 40, replace=False)
    offs[bad[:20]] = buf.size + rng.integers(0, 1000, 20)
    lens[bad[20:]] = (buf.size - offs[bad[20:]] + rng.integers(1, 50, 20)).astype(np.uint32)
    rec_off = np.where(offs > buf.size, 0, offs)
    rec_len = np.where((offs > buf.size) | (offs + lens > buf.size), 0, lens).astype(np.uint32)
    want = coracle.checksum_slices(buf, rec_off, rec_len, skips)
    d = to_dev(buf)
    do, dl, ds = to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)), to_dev(skips.astype(np.int32))
    got = lp.checksum_slices(d, do, dl, ds).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, want)
    protos = rng.integers(0, 256, n, dtype=np.uint8)
    for fn, alen, ofn in ((lp.ipv4_checksum_slices, 8, coracle.ipv4_checksum),
                          (lp.ipv6_checksum_slices, 32, coracle.ipv6_checksum)):
        raw = rng.integers(0, 256, n * alen + 1, dtype=np.uint8)
        for shift in (0, 1):                    # the addrs array 4-B aligned, then at an odd address
            a_dev = to_dev(raw)[shift:shift + n * alen].view(n, alen)
            a = raw[shift:shift + n * alen].reshape(n, alen)
            got = fn(d, do, dl, ds, a_dev, to_dev(protos)).cpu().numpy().view(np.uint16)
            h = alen // 2
            for i in list(range(0, n, 41)) + [int(x) for x in bad]:
                o, ln = int(rec_off[i]), int(rec_len[i])
                assert got[i] == ofn(bytes(buf[o:o + ln]), int(skips[i]), b"", bytes(a[i, :h]), bytes(a[i, h:]),
                                     int(protos[i])), (alen, shift, i)


@pytest.mark.parametrize("kernel", ["run", "group"])
@pytest.mark.parametrize("short", [False, True])
def test_random_adv_slices_vs_oracle(kernel, short, tune):
    """*_checksum_adv (extra_data) batched: main and extra slices at every byte
    alignment, odd/even/empty extras, extras longer than one 16-lane pass; short
    main and extra slices (0-100 B: own-lane, 2- and 4-lane classes of
    slice_run_kernel, its extra range a second pass), both slice kernels."""
    tune("slice_kernel", kernel)
    rng = np.random.default_rng(23 + short)
    n = 6000
    buf = rng.integers(0, 256, 1 << 21, dtype=np.uint8)
    lens = rng.integers(0, 101 if short else 1600, n).astype(np.uint32)
    offs = rng.integers(0, buf.size - 1700, n).astype(np.uint64)
    skips = rng.integers(0, 60 if short else 900, n).astype(np.uint32)
    elens = rng.integers(0, 101 if short else 600, n).astype(np.uint32)
    elens[::5] = rng.integers(0, 4, elens[::5].size)
    elens[1::5] = 0
    eoffs = rng.integers(0, buf.size - 700, n).astype(np.uint64)
    addrs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    protos = rng.integers(0, 256, n, dtype=np.uint8)
    for version, alen, ofn in ((4, 8, coracle.ipv4_checksum), (6, 32, coracle.ipv6_checksum)):
        a = np.ascontiguousarray(addrs[:, :alen])
        got = lp.checksum_adv_slices(version, to_dev(buf), to_dev(offs.astype(np.int64)),
                                     to_dev(lens.astype(np.int32)), to_dev(skips.astype(np.int32)),
                                     to_dev(eoffs.astype(np.int64)), to_dev(elens.astype(np.int32)),
                                     to_dev(a), to_dev(protos)).cpu().numpy().view(np.uint16)
        h = alen // 2
        for i in range(0, n, 7):
            o, ln, eo, el = int(offs[i]), int(lens[i]), int(eoffs[i]), int(elens[i])
            want = ofn(bytes(buf[o:o + ln]), int(skips[i]), bytes(buf[eo:eo + el]), bytes(a[i, :h]),
                       bytes(a[i, h:]), int(protos[i]))
            assert got[i] == want, (version, i, ln, el, o % 16, eo % 16)


@pytest.mark.parametrize("kernel", ["run", "group"])
def test_adv_slices_match_tcp_with_options_split(kernel, tune):
    """A TCP segment checksummed whole equals the same segment split into a
    header slice + an even-length extra (the way tcp::ipv4_checksum_adv is used
    to checksum a header and a separately held payload)."""
    tune("slice_kernel", kernel)
    rng = np.random.default_rng(5)
    seg = rng.integers(0, 256, 1000, dtype=np.uint8)
    buf = np.concatenate([np.zeros(3, np.uint8), seg, np.zeros(64, np.uint8)])
    src, dst = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    addrs = np.frombuffer(src + dst, np.uint8).reshape(1, 8)
    whole = coracle.ipv4_checksum(seg.tobytes(), 8, b"", src, dst, 6)
    for hl in (20, 32, 60):
        got = lp.checksum_adv_slices(4, to_dev(buf), to_dev(np.array([3], np.int64)), to_dev(np.array([hl], np.int32)),
                                     to_dev(np.array([8], np.int32)), to_dev(np.array([3 + hl], np.int64)),
                                     to_dev(np.array([1000 - hl], np.int32)), to_dev(addrs),
                                     to_dev(np.array([6], np.uint8)))
        assert int(got.cpu().numpy().view(np.uint16)[0]) == whole, hl


def test_maximum_sizes_all_ones():
    """The largest sums the path can meet: IPv4 total_length 65535 and IPv6
    payload_length 65535 frames of 0xFF bytes (every 16-bit word 0xFFFF), plus
    the same through the fixed-stride jumbo kernel, and util::checksum slices
    of 0xFF up to 131070 bytes (the longest slice whose u32 word sum cannot wrap,
    SURVEY.md §8(a) a1)."""
    rng = np.random.default_rng(77)
    frames = []
    for kind in ("udp", "tcp", "udp6", "tcp6"):
        iphl = 40 if kind.endswith("6") else 20
        f = bytearray(framegen.build_frame(rng, kind, 65535 - (0 if iphl == 40 else 20)))
        f[14 + iphl:] = b"\xff" * (len(f) - 14 - iphl)
        frames.append(bytes(f))
        g = bytearray(f)
        g[14 + iphl + 100] = 0          # one zero byte: a different sum
        frames.append(bytes(g))
    buf, offs, lens = framegen.pack(frames, gap=15, rng=rng)
    rec = oracle_desc(buf, offs, lens)
    compare(run_desc(buf, offs, lens), rec)
    # the same frames through the fixed-stride kernels (one frame length at a time)
    for f in frames[:2]:
        stride = len(f) + 3
        sbuf = np.zeros(stride * 4 + 64, np.uint8)
        for i in range(4):
            sbuf[i * stride:i * stride + len(f)] = np.frombuffer(f, np.uint8)
        srec = coracle.rx_batch(sbuf, 4, stride=stride, frame_len=len(f))
        res = lp.rx_process(to_dev(sbuf), stride=stride, frame_len=len(f), n_frames=4, columns=ALL_COLUMNS)
        torch.cuda.synchronize()
        compare(res, srec)
    # util::checksum over long all-ones slices at every alignment
    big = np.full(131070 + 64, 0xFF, np.uint8)
    offs_s = np.array([0, 1, 2, 7, 15, 3, 0], np.int64)
    lens_s = np.array([131070, 131069, 131068, 65535, 100000, 131000, 1], np.int32)
    skips = np.array([0, 5, 70000, 65534, 3, 1 << 20, 0], np.int32)
    want = coracle.checksum_slices(big, offs_s.astype(np.uint64), lens_s.astype(np.uint32), skips.astype(np.uint32))
    got = lp.checksum_slices(to_dev(big), to_dev(offs_s), to_dev(lens_s), to_dev(skips))
    assert np.array_equal(got.cpu().numpy().view(np.uint16), want)


def test_packed_result_block_to_host():
    """RxResult keeps counters + columns in one block; to_host moves them in one
    copy and the host bytes hold exactly the device columns."""
    rng = np.random.default_rng(12)
    frames = framegen.random_frames(rng, 3000)
    buf, offs, lens = framegen.pack(frames, gap=4, rng=rng)
    res = run_desc(buf, offs, lens)
    host = res.to_host()
    torch.cuda.synchronize()
    h = host.numpy()
    base = res.block.data_ptr()
    for c, t in res.columns.items():
        o = t.data_ptr() - base
        assert o % 256 == 0
        got = h[o:o + t.numel() * t.element_size()].view(COLUMNS[c][1]).reshape(t.shape)
        assert np.array_equal(got, t.cpu().numpy().view(COLUMNS[c][1]))
    assert np.array_equal(h[:64].view(np.uint64), res.counters.cpu().numpy().view(np.uint64))
    compare(res, oracle_desc(buf, offs, lens))


def test_concurrent_contexts_from_host_threads():
    """Header contract: distinct contexts are independent. Four host threads,
    each with its own context and stream, process different batches at once
    (ctypes releases the GIL inside the C-ABI call): every record bit-exact."""
    import threading
    rng = np.random.default_rng(21)
    jobs = []
    for t in range(4):
        frames = framegen.random_frames(rng, 2500, max_len=3000)
        buf, offs, lens = framegen.pack(frames, gap=t, rng=rng)
        jobs.append((buf, offs, lens, oracle_desc(buf, offs, lens)))
    results, errors = [None] * 4, []

    def work(t):
        try:
            buf, offs, lens, _ = jobs[t]
            ctx = lp.engine.Context(0)
            s = torch.cuda.Stream(DEV)
            with torch.cuda.stream(s):
                d, o, ln = to_dev(buf), to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32))
                for _ in range(5):
                    res = lp.rx_process(d, offsets=o, lengths=ln, columns=ALL_COLUMNS, stream=s, ctx=ctx)
            s.synchronize()
            results[t] = res
        except Exception as e:                    # surfaced below
            errors.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for t in range(4):
        compare(results[t], jobs[t][3])


@pytest.mark.parametrize("kind", ["udp64", "tcp1500"])
def test_batches_past_4gib(kind):
    """64-bit addressing: a 4.5-5 GiB fixed-stride batch (the 1-GiB-class synth
    batch tiled on the device) — counters are the tile's times the tile count,
    and the records of the frames past 4 GiB equal the oracle's for their
    source frames; then a descriptor batch whose frames all sit past 4 GiB."""
    n0 = {"udp64": 1 << 24, "tcp1500": 1 << 20}[kind]
    w = lp.synth.make(kind, n0, seed=3, corrupt_ppm=10000)
    tile = torch.from_numpy(w.buf[: n0 * w.stride]).to(DEV)
    reps = 5 if kind == "udp64" else 3
    big = torch.cat([tile] * reps + [torch.zeros(64, dtype=torch.uint8, device=DEV)])
    n = n0 * reps
    assert n * w.stride > (1 << 32) + (1 << 28)
    res = lp.rx_process(big, stride=w.stride, frame_len=w.frame_len, n_frames=n, columns=IPV4_COLS_ALL)
    torch.cuda.synchronize()
    c = res.counter_dict()
    assert c["frames"] == n and c["ip_csum_bad"] == reps * w.expect["ip_bad"]
    assert c["l4_csum_bad"] == reps * w.expect["l4_bad"] and c["bytes"] == reps * w.expect["bytes"]
    k = 1 << 14                                    # the last k frames: all past 4 GiB
    src0 = n0 - k
    rec = coracle.rx_batch(w.buf[src0 * w.stride:(src0 + k) * w.stride + 64], k, stride=w.stride,
                           frame_len=w.frame_len)
    got = {col: t[n - k:].cpu().numpy().view(COLUMNS[col][1]) for col, t in res.columns.items()}
    for col, v in got.items():
        assert np.array_equal(v, rec[col]), col
    # descriptor mode, every frame past 4 GiB (offsets > 2^32)
    first = n - k
    offs = (torch.arange(k, dtype=torch.int64, device=DEV) + first) * w.stride
    lens = torch.full((k,), w.frame_len, dtype=torch.int32, device=DEV)
    assert int(offs[0]) > (1 << 32)
    res2 = lp.rx_process(big, offsets=offs, lengths=lens, columns=IPV4_COLS_ALL)
    torch.cuda.synchronize()
    for col, t in res2.columns.items():
        assert np.array_equal(t.cpu().numpy().view(COLUMNS[col][1]), rec[col]), col
    del big, tile, res, res2
    torch.cuda.empty_cache()


IPV4_COLS_ALL = lp.IPV4_COLUMNS


def test_empty_batches():
    """n_frames == 0 is a no-op in every mode (no launch, counters untouched)."""
    d = torch.zeros(64, dtype=torch.uint8, device=DEV)
    e64 = torch.zeros(0, dtype=torch.int64, device=DEV)
    e32 = torch.zeros(0, dtype=torch.int32, device=DEV)
    res = lp.rx_process(d, offsets=e64, lengths=e32, columns=ALL_COLUMNS)
    res2 = lp.rx_process(d, stride=64, frame_len=64, n_frames=0, columns=ALL_COLUMNS)
    lp.tx_fill_checksums(d, stride=64, frame_len=64, n_frames=0)
    torch.cuda.synchronize()
    assert res.counter_dict()["frames"] == 0 and res2.counter_dict()["frames"] == 0
    assert int(d.sum()) == 0


def test_last_rx_kernel_names_the_launched_instantiation():
    """pnetgpu_last_rx_kernel: the instantiation rocprofv3 reports for each batch shape."""
    w = lp.synth.make("udp64", 4096, seed=3)
    lp.rx_process(to_dev(w.buf), stride=64, frame_len=64, n_frames=4096)
    assert lp.last_rx_kernel() == "rx_small_kernel<false, false>"
    lp.rx_process(to_dev(w.buf), stride=64, frame_len=64, n_frames=4096, columns=("status", "tcp_flags"))
    assert lp.last_rx_kernel() == "rx_small_kernel<false, true>"
    w = lp.synth.make("imix", 2048, seed=3)
    d = to_dev(w.buf)
    lp.rx_process(d, offsets=to_dev(w.offsets.astype(np.int64)), lengths=to_dev(w.lengths.astype(np.int32)))
    assert re.fullmatch(SHAPE_RE["mixed"] + "false, false>", lp.last_rx_kernel())
    lp.tx_fill_checksums(d, offsets=to_dev(w.offsets.astype(np.int64)), lengths=to_dev(w.lengths.astype(np.int32)))
    assert re.fullmatch(SHAPE_RE["mixed"] + "false, true>", lp.last_rx_kernel())
    w = lp.synth.make("tcp1500", 256, seed=3)
    lp.rx_process(to_dev(w.buf), stride=1500, frame_len=1500, n_frames=256)
    assert re.fullmatch(SHAPE_RE["mtu"] + "false, false>", lp.last_rx_kernel())
    torch.cuda.synchronize()


# ---- util::checksum over uniform slices (pnetgpu_checksum_slices_strided) ----

def _strided_want(buf, n, first, stride, slen, skip):
    offs = first + np.arange(n, dtype=np.uint64) * np.uint64(stride)
    return coracle.checksum_slices(buf, offs, np.full(n, slen, np.uint32), np.full(n, skip, np.uint32))


def test_strided_slices_reference_bench_shapes():
    """checksum_benchmarks.rs:8-18: util::checksum(&[99u8; 20], 5) and
    util::checksum(&[123u8; 1024], 5), batched back to back without descriptors."""
    for fill, size, n in ((99, 20, 100003), (123, 1024, 2049)):
        buf = np.full(n * size + 32, fill, np.uint8)
        got = lp.checksum_slices_strided(to_dev(buf), n, size, size, 5).cpu().numpy().view(np.uint16)
        want = coracle.checksum(bytes([fill] * size), 5)
        assert (got == want).all(), (size, want)


@pytest.mark.parametrize("stride,slen", [(20, 20), (0, 7), (1, 64), (7, 20), (16, 16), (63, 64), (64, 64),
                                         (64, 1), (65, 20), (100, 256), (300, 257), (1024, 1000), (40, 0),
                                         (19, 18), (21, 21), (62, 62), (64, 63), (3, 3), (40, 35)])
def test_strided_slices_random_vs_oracle(stride, slen):
    rng = np.random.default_rng(stride * 1000 + slen)
    n = 5000
    for first, data_off, skip in ((0, 0, 5), (13, 3, 0), (7, 6, 40), (2, 1, 1 << 20)):
        total = first + (n - 1) * stride + slen
        buf = rng.integers(0, 256, total, dtype=np.uint8)
        full = to_dev(np.concatenate([np.zeros(16, np.uint8), buf, np.zeros(64, np.uint8)]))
        d = full[16 + data_off:16 + total]                    # buf[data_off:] at a misaligned device pointer
        got = lp.checksum_slices_strided(d, n, stride, slen, skip, first_offset=first - data_off)
        want = _strided_want(buf[data_off:], n, first - data_off, stride, slen, skip)
        assert np.array_equal(got.cpu().numpy().view(np.uint16), want), (first, data_off, skip)


def test_strided_slices_bounds_are_checked():
    d = to_dev(np.zeros(1000, np.uint8))
    with pytest.raises(lp.PnetGpuError):
        lp.checksum_slices_strided(d, 11, 100, 1, 0)        # slice 10 starts at byte 1000
    with pytest.raises(lp.PnetGpuError):
        lp.checksum_slices_strided(d, 1, 0, 1001, 0)
    out = lp.checksum_slices_strided(d, 10, 100, 100, 0)      # exactly fits
    assert (out.cpu().numpy().view(np.uint16) == 0xFFFF).all()   # finalize(0) of non-empty zero slices
    assert lp.checksum_slices_strided(d, 0, 100, 100, 0).numel() == 0


def test_strided_slices_random_shapes_fuzz():
    """400 random uniform-slice batches (stride 0-300, length 0-300, first offset,
    data-pointer misalignment, skipword in or past the slice), each against the
    oracle: every kernel the strided entry point can pick."""
    rng = np.random.default_rng(2024)
    for _ in range(400):
        stride = int(rng.integers(0, 301))
        slen = int(rng.integers(0, 301))
        n = int(rng.integers(1, 700))
        first = int(rng.integers(0, 40))
        mis = int(rng.integers(0, 16))
        skip = int(rng.integers(0, slen // 2 + 3))
        total = first + (n - 1) * stride + slen
        buf = rng.integers(0, 256, max(total, 1), dtype=np.uint8)
        full = to_dev(np.concatenate([np.zeros(16, np.uint8), buf, np.zeros(64, np.uint8)]))
        d = full[16 + mis:16 + max(total, mis)]
        if first < mis:
            continue
        got = lp.checksum_slices_strided(d, n, stride, slen, skip, first_offset=first - mis)
        want = _strided_want(buf[mis:], n, first - mis, stride, slen, skip)
        assert np.array_equal(got.cpu().numpy().view(np.uint16), want), (stride, slen, n, first, mis, skip)


# ---- util::checksum over compact (8-B) slice descriptors ----

def test_compact_slices_kats_and_random_vs_oracle():
    """pnetgpu_checksum_slices_compact: the util.rs / icmp.rs KAT slices at six
    misalignments, and 20,000 random slices (0..2000 B, any alignment, skipword
    inside / at the edge of / past the slice, gaps and overlaps) through both
    slice kernels, against the oracle."""
    vs = kats.by_kind("sum_be_words", "checksum")
    for misalign in (0, 1, 2, 3, 5, 15):
        parts, offs, lens, skips, want = [], [], [], [], []
        pos = 0
        for v in vs:
            pad = (misalign - pos) % 16
            parts.append(bytes(pad))
            pos += pad
            offs.append(pos)
            lens.append(len(v["data"]))
            skips.append(v["skipword"])
            parts.append(v["data"])
            pos += len(v["data"])
            want.append(v["expected"] if v["kind"] == "checksum" else
                        (pyoracle.finalize(v["expected"]) if v["data"] else 0))
        buf = np.frombuffer(b"".join(parts) + bytes(32), dtype=np.uint8)
        desc = lp.slice_descriptors(offs, lens, skips, device=DEV)
        got = lp.checksum_slices_compact(to_dev(buf), desc).cpu().numpy().view(np.uint16)
        assert list(got) == want, misalign
    rng = np.random.default_rng(77)
    buf = rng.integers(0, 256, 3 << 20, dtype=np.uint8)
    n = 20000
    lens = rng.integers(0, 2001, n).astype(np.uint32)
    lens[rng.random(n) < 0.5] %= 64                       # mostly short, as packets' headers are
    offs = rng.integers(0, buf.size - 2001, n).astype(np.uint64)
    skips = np.where(rng.random(n) < 0.8, rng.integers(0, 40, n), rng.integers(0, 1200, n)).astype(np.uint32)
    want = coracle.checksum_slices(buf, offs, lens, skips)
    desc = lp.slice_descriptors(offs, lens, skips, device=DEV)
    d = to_dev(np.concatenate([buf, np.zeros(32, np.uint8)]))[: buf.size]
    for kern in ("run", "group", "tiny"):
        with lp.engine.tuning(0, slice_kernel=kern):
            got = lp.checksum_slices_compact(d, desc).cpu().numpy().view(np.uint16)
        assert np.array_equal(got, want), kern
    big = np.full(70000, 7, np.uint8)                     # the compact maximum: 65535-B slices
    desc = lp.slice_descriptors([0, 1, 4465], [65535, 65535, 65535], [0, 3, 32767], device=DEV)
    got = lp.checksum_slices_compact(to_dev(big), desc).cpu().numpy().view(np.uint16)
    want = coracle.checksum_slices(big, np.array([0, 1, 4465], np.uint64), np.full(3, 65535, np.uint32),
                                   np.array([0, 3, 32767], np.uint32))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("span", ["0", None])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_dense_runs_of_packed_slices(seed, span, tune):
    """slice_run_kernel's dense-run path: runs of 64 sorted small slices packed
    in a span of at most 5 KiB arrive as coalesced loads into LDS. Packed
    slices (0..64 B, gaps 0..k), every alignment, and runs that must fall back
    to per-lane gathers: one slice out of order, a span just past 5 KiB, lane
    0 or the last lane empty, a slice past the buffer, a slice ending after
    the last one's end, a final partial run. Full and compact descriptors,
    ipv4/ipv6 pseudo-header forms, against the oracle; with every eligible run
    staged (slice_dense_span 0) and with the default span threshold."""
    if span is not None:
        tune("slice_dense_span", int(span))
    tune("slice_kernel", "run")
    rng = np.random.default_rng(900 + seed)
    n = 64 * 200 + 23
    maxgap = (0, 4, 20)[seed]
    lens = rng.integers(0, 65, n).astype(np.uint32)
    gaps = rng.integers(0, maxgap + 1, n)
    offs = (np.cumsum(lens.astype(np.int64) + gaps) - lens - gaps + int(rng.integers(0, 16))).astype(np.uint64)
    runs = n // 64
    for r in rng.choice(runs, 40, replace=False):         # break the dense condition in some runs
        b = 64 * int(r)
        kind = int(rng.integers(0, 6))
        if kind == 0:
            offs[b + 10], offs[b + 30] = offs[b + 30], offs[b + 10]
        elif kind == 1:
            lens[b + 63] = 0
        elif kind == 2:
            lens[b] = 0
        elif kind == 3:
            lens[b + 5] = 64
            offs[b + 5] = offs[b + 63] + 10
        elif kind == 4:
            offs[b + 63] = int(offs[b]) + 5120 - int(lens[b + 63]) + int(rng.integers(-2, 3))
        else:
            offs[b + 20] = 1 << 40
    size = int(max(o + l for o, l in zip(offs, lens) if o < (1 << 40))) + 7
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    lens[-1] = 3
    offs[-1] = size - 3                                    # the very last bytes of the buffer
    skips = np.where(rng.random(n) < 0.7, rng.integers(0, 34, n), rng.integers(0, 100, n)).astype(np.uint32)
    bad = offs > size
    rec_off = np.where(bad, 0, offs)
    rec_len = np.where(bad, 0, lens).astype(np.uint32)
    want = coracle.checksum_slices(buf, rec_off, rec_len, skips)
    d = to_dev(np.concatenate([buf, np.zeros(32, np.uint8)]))[:size]
    do, dl, ds = to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)), to_dev(skips.astype(np.int32))
    got = lp.checksum_slices(d, do, dl, ds).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, want)
    ok = ~bad
    desc = lp.slice_descriptors(rec_off[ok], rec_len[ok], skips[ok], device=DEV)
    got = lp.checksum_slices_compact(d, desc).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, want[ok])
    protos = rng.integers(0, 256, n, dtype=np.uint8)
    for fn, alen, ofn in ((lp.ipv4_checksum_slices, 8, coracle.ipv4_checksum),
                          (lp.ipv6_checksum_slices, 32, coracle.ipv6_checksum)):
        a = rng.integers(0, 256, (n, alen), dtype=np.uint8)
        got = fn(d, do, dl, ds, to_dev(a), to_dev(protos)).cpu().numpy().view(np.uint16)
        h = alen // 2
        for i in list(range(0, n, 37)) + list(np.nonzero(bad)[0]):
            o, ln = int(rec_off[i]), int(rec_len[i])
            assert got[i] == ofn(bytes(buf[o:o + ln]), int(skips[i]), b"", bytes(a[i, :h]), bytes(a[i, h:]),
                                 int(protos[i])), (alen, i)


@pytest.mark.parametrize("kernel", ["run", "tiny"])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_runs_of_small_slices_vs_oracle(seed, kernel, tune):
    """slice_run_kernel on runs whose 64 slices are all small (each summed by its
    own lane): short slices at every alignment with the skipped word inside /
    straddling / past the slice, empty and out-of-bounds descriptors, batch
    sizes giving an odd run count with a ragged last run, a long slice every few
    hundred slices (its run takes the group path), and packed 64-B runs (dense)
    between them; 16-B and compact descriptors, against the oracle. (Written
    for a two-runs-at-once variant, measured slower and not kept:
    profiles/r03/slices/ab_run_pairs.txt.) slice_tiny_kernel too: its own
    lanes sum slices of at most 3 granules, the long ones go to its wave loop."""
    tune("slice_kernel", kernel)
    rng = np.random.default_rng(900 + seed)
    n = 64 * (201 + 2 * seed) + 13 + seed
    buf = rng.integers(0, 256, 1 << 21, dtype=np.uint8)
    lens = rng.integers(0, 50, n).astype(np.uint32)
    lens[rng.random(n) < 0.02] = 0
    offs = rng.integers(0, buf.size - 6000, n).astype(np.uint64)
    if seed != 2:                                       # seed 2: every run qualifies
        big = rng.choice(n, n // 400, replace=False)
        lens[big] = rng.integers(70, 5000, big.size)
    r = 64 * (30 + seed)                                # two packed 64-B runs: dense, not paired
    offs[r:r + 128] = 4096 + 64 * np.arange(128, dtype=np.uint64)
    lens[r:r + 128] = 64
    skips = np.where(rng.random(n) < 0.7, rng.integers(0, 26, n), rng.integers(0, 3000, n)).astype(np.uint32)
    bad = rng.choice(n, 30, replace=False)
    offs[bad[:15]] = buf.size + rng.integers(0, 1000, 15)
    lens[bad[15:]] = (buf.size - offs[bad[15:]] + rng.integers(1, 40, 15)).astype(np.uint32)
    rec_off = np.where(offs > buf.size, 0, offs)
    rec_len = np.where((offs > buf.size) | (offs + lens > buf.size), 0, lens).astype(np.uint32)
    want = coracle.checksum_slices(buf, rec_off, rec_len, skips)
    d = to_dev(buf)
    got = lp.checksum_slices(d, to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)),
                             to_dev(skips.astype(np.int32))).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, want)
    co, cl, cs = offs, np.minimum(lens, 0xFFFF), np.minimum(skips, 0xFFFF)   # compact: u32 offset, u16 length
    desc = lp.slice_descriptors(co, cl, cs, device=DEV)
    got = lp.checksum_slices_compact(d, desc).cpu().numpy().view(np.uint16)
    c_len = np.where((co > buf.size) | (co + cl > buf.size), 0, cl).astype(np.uint32)
    want_c = coracle.checksum_slices(buf, np.where(co > buf.size, 0, co), c_len, cs.astype(np.uint32))
    assert np.array_equal(got, want_c)


@pytest.mark.parametrize("compact", [False, True])
def test_tiny_kernel_reference_shape_and_choice(compact):
    """slice_tiny_kernel (software-pipelined runs of 64 slices): the reference's
    20-B util::checksum bench shape (checksum_benchmarks.rs:8-12) packed back
    to back with random bytes, skipword 5, at every start alignment, with a
    ragged last run, through the default choice (<= 32 buffer bytes per slice
    takes the tiny kernel: pnetgpu_last_rx_kernel names it); then slices of
    0..33 B at any alignment with the skipped word anywhere (its two bytes
    read from the granule registers: inside, straddling the end, past it),
    each slice's neighbours overlapping, and a few long slices (the wave loop)
    in a buffer still <= 32 B per slice. Against the oracle."""
    rng = np.random.default_rng(31 + compact)
    for first in (0, 1, 7, 15):
        n = 64 * 411 + 37
        buf = rng.integers(0, 256, first + 20 * n, dtype=np.uint8)
        offs = first + 20 * np.arange(n, dtype=np.uint64)
        lens = np.full(n, 20, np.uint32)
        skips = np.full(n, 5, np.uint32)
        want = coracle.checksum_slices(buf, offs, lens, skips)
        d = to_dev(np.concatenate([buf, np.zeros(32, np.uint8)]))[: buf.size]
        if compact:
            got = lp.checksum_slices_compact(d, lp.slice_descriptors(offs, lens, skips, device=DEV))
        else:
            got = lp.checksum_slices(d, to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)),
                                     to_dev(skips.astype(np.int32)))
        assert lp.last_rx_kernel() == f"slice_tiny_kernel<{'true' if compact else 'false'}>"
        assert np.array_equal(got.cpu().numpy().view(np.uint16), want), first
    n = 64 * 700 + 5
    buf = rng.integers(0, 256, 32 * n, dtype=np.uint8)
    lens = rng.integers(0, 34, n).astype(np.uint32)
    offs = rng.integers(0, buf.size - 6000, n).astype(np.uint64)
    skips = np.where(rng.random(n) < 0.8, rng.integers(0, 18, n), rng.integers(0, 70000, n)).astype(np.uint32)
    big = rng.choice(n, 40, replace=False)
    lens[big] = rng.integers(34, 5000, big.size)
    skips[big[:20]] = rng.integers(0, 2500, 20)
    if compact:
        skips = np.minimum(skips, 0xFFFF)
    want = coracle.checksum_slices(buf, offs, lens, skips)
    d = to_dev(buf)
    if compact:
        got = lp.checksum_slices_compact(d, lp.slice_descriptors(offs, lens, skips, device=DEV))
    else:
        got = lp.checksum_slices(d, to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)),
                                 to_dev(skips.astype(np.int32)))
    assert lp.last_rx_kernel().startswith("slice_tiny_kernel")
    assert np.array_equal(got.cpu().numpy().view(np.uint16), want)


def run_desc_form(buf, offs, lens, compact, columns=RECORD_COLUMNS):
    """rx_process over full (u64/u32) or compact (u32/u16) descriptors."""
    if not compact:
        return run_desc(buf, offs, lens, columns=columns)
    res = lp.rx_process(to_dev(buf), offsets=to_dev(np.asarray(offs, np.uint32).view(np.int32)),
                        lengths=to_dev(np.asarray(lens, np.uint16).view(np.int16)), columns=columns,
                        flags=lp.DESC_COMPACT)
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("seed", [0, 1])
def test_descriptor_runs_of_short_frames(seed, compact):
    """The mixed kernel's short-run path (every frame of a run at most 64 B: the
    small kernel's register fast path on frames realigned from their slots):
    random UDP/TCP/ICMP/IPv6 frames of 0-64 B, the <= 64-B edge frames (IHL
    0-15, short L4, IPv6), a ragged last run; then the same batch with a few
    frames moved off alignment, one 65-B frame and invalid descriptors (their
    runs take the generic parse). Every record column and the counters equal
    the oracle's, with full (12-B) and compact (6-B, the ring's and the
    bench's IMIX form) descriptors."""
    rng = np.random.default_rng(1300 + seed)
    edge = [f for f in framegen.edge_frames(rng) if len(f) <= 64]
    frames = framegen.random_frames(rng, 64 * 90 + 37, min_len=0, max_len=64)
    frames[100:100 + len(edge)] = edge
    buf, offs, lens = framegen.pack(frames, align=16)
    rec = oracle_desc(buf, offs, lens)
    res = run_desc_form(buf, offs, lens, compact)
    compare(res, rec)
    assert res.counter_dict() == oracle_counters(rec, lens)
    # some runs no longer qualify: a misaligned frame, a 65-B frame, bad descriptors
    f65 = np.frombuffer(bytes(framegen.random_frames(rng, 1, min_len=65, max_len=65)[0]), np.uint8)
    buf2 = np.concatenate([buf, f65, np.zeros(32, np.uint8)])
    offs2, lens2 = offs.copy(), lens.copy()
    offs2[64 * 3 + 5] += 1
    lens2[64 * 3 + 5] = min(int(lens2[64 * 3 + 5]), 15)
    offs2[64 * 7 + 9], lens2[64 * 7 + 9] = buf.size, 65
    offs2[64 * 11] = buf2.size + 64
    if compact:                                          # a length running past the end, in 16 bits
        offs2[64 * 13 + 63], lens2[64 * 13 + 63] = buf2.size - 10, 65
    else:
        lens2[64 * 13 + 63] = buf2.size
    rec2 = oracle_desc(buf2, offs2, lens2)
    assert (rec2["status"][[64 * 11, 64 * 13 + 63]] & pyoracle.ST_DESC_INVALID).all()
    res2 = run_desc_form(buf2, offs2, lens2, compact)
    compare(res2, rec2)
    assert res2.counter_dict() == oracle_counters(rec2, lens2)
    # any alignment: frames straddling four or five granules, runs of both kinds
    for align, gap in ((1, 0), (1, 7), (4, 0)):
        buf3, offs3, lens3 = framegen.pack(frames, align=align, gap=gap, rng=rng)
        rec3 = oracle_desc(buf3, offs3, lens3)
        res3 = run_desc_form(buf3, offs3, lens3, compact)
        compare(res3, rec3)
        assert res3.counter_dict() == oracle_counters(rec3, lens3)


def test_slice_argument_validation():
    """The slice entry points refuse arrays the kernels would misread (host
    pointers, other dtypes, short arrays) and u32 arguments that would be
    truncated, before any launch; compact descriptors on the host are copied
    to the data's device (slice_descriptors' default) and give the same sums."""
    rng = np.random.default_rng(31)
    buf = rng.integers(0, 256, 4096, dtype=np.uint8)
    d = to_dev(buf)
    offs, lens, skips = np.arange(0, 4000, 100, dtype=np.uint64), np.full(40, 60, np.uint32), np.full(40, 2, np.uint32)
    want = coracle.checksum_slices(buf, offs, lens, skips)
    host_desc = lp.slice_descriptors(offs, lens, skips)                  # a CPU tensor
    assert not host_desc.is_cuda
    assert np.array_equal(lp.checksum_slices_compact(d, host_desc).cpu().numpy().view(np.uint16), want)
    with pytest.raises(TypeError):
        lp.checksum_slices_compact(d, host_desc.int())
    do, dl, ds = to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)), to_dev(skips.astype(np.int32))
    assert np.array_equal(lp.checksum_slices(d, do, dl, ds).cpu().numpy().view(np.uint16), want)
    with pytest.raises(TypeError):
        lp.checksum_slices(d, do.cpu(), dl, ds)
    with pytest.raises(TypeError):
        lp.checksum_slices(d, do, dl.long(), ds)
    with pytest.raises(ValueError):
        lp.checksum_slices(d, do, dl[:10], ds)
    with pytest.raises(ValueError):
        lp.ipv4_checksum_slices(d, do, dl, ds, to_dev(np.zeros((40, 4), np.uint8)), to_dev(np.zeros(40, np.uint8)))
    for kw in ({"stride": 1 << 32}, {"slice_len": 1 << 32}, {"skipword": -1}):
        args = {"stride": 20, "slice_len": 20, "skipword": 5, **kw}
        with pytest.raises(ValueError):
            lp.checksum_slices_strided(d, 10, args["stride"], args["slice_len"], args["skipword"])


# ---- descriptor batches with a frame-size hint (PNETGPU_DESC_HINT_*) --------

_HINT_KERNEL = {0: SHAPE_RE["mixed"], "large": SHAPE_RE["mtu"], "jumbo": SHAPE_RE["jumbo"]}


@pytest.mark.parametrize("hint", [0, "large", "jumbo"])
@pytest.mark.parametrize("rxflags", [0, "vlan_ext"])
def test_descriptor_size_hints_any_batch(hint, rxflags):
    """A size hint only picks the tail shape: any descriptor batch (random and
    malformed frames up to 9,100 B, IPv6, VLAN tags and extension headers, at
    any alignment, full and compact descriptors) under either hint gives the
    oracle's records and counters, receive and TX fill alike, and the launch
    names the hinted instantiation."""
    fl = {0: 0, "large": lp.DESC_HINT_LARGE, "jumbo": lp.DESC_HINT_JUMBO}[hint]
    rx = 0 if not rxflags else lp.engine.RX_VLAN | lp.engine.RX_IPV6_EXT
    rng = np.random.default_rng(900 + fl + rx)
    frames = framegen.edge_frames(rng) + framegen.random_frames(rng, 3000, max_len=9100)
    buf, offs, lens = framegen.pack(frames, gap=11, rng=rng)
    rec = coracle.rx_batch(buf, len(offs), offsets=offs, lengths=lens, flags=rx, nthreads=NTHREADS)
    d = to_dev(buf)
    o32 = to_dev(offs.astype(np.uint32).view(np.int32))
    l16 = to_dev(lens.astype(np.uint16).view(np.int16))
    for compact in (False, True):
        o, ln = (o32, l16) if compact else (to_dev(offs.astype(np.int64)), to_dev(lens.astype(np.int32)))
        res = lp.rx_process(d, offsets=o, lengths=ln, columns=ALL_COLUMNS,
                            flags=fl | rx | (lp.DESC_COMPACT if compact else 0))
        torch.cuda.synchronize()
        compare(res, rec)
        assert res.counter_dict() == oracle_counters(rec, lens), (hint, compact)
        assert re.match(_HINT_KERNEL[hint], lp.last_rx_kernel()), lp.last_rx_kernel()
    # TX fill under the hint: the patched buffer equals the oracle's
    dt = to_dev(buf.copy())
    lp.tx_fill_checksums(dt, offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                         flags=fl | rx)
    want_buf, _ = coracle.tx_fill(buf, len(offs), offsets=offs, lengths=lens, flags=rx)
    torch.cuda.synchronize()
    assert np.array_equal(dt.cpu().numpy(), want_buf)


def test_hints_on_the_bench_batches():
    """The hint the rule picks for each workload's lengths, and the records
    under it: 1500-B UDP frames as a descriptor batch (LARGE -> the MTU shape),
    9000-B IPv6 frames (JUMBO), IMIX (no hint)."""
    for name, n, want in (("udp1500", 1 << 14, lp.DESC_HINT_LARGE), ("udp6_jumbo", 1 << 11, lp.DESC_HINT_JUMBO),
                          ("imix", 1 << 16, 0)):
        w = lp.synth.make(name, n, seed=17, corrupt_ppm=20000)
        if w.stride:
            offs = np.arange(n, dtype=np.uint64) * np.uint64(w.stride)
            lens = np.full(n, w.frame_len, np.uint32)
        else:
            offs, lens = w.offsets, w.lengths
        hint = lp.desc_size_hint(lens)
        assert hint == want, name
        res = lp.rx_process(to_dev(w.buf), offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)),
                            flags=hint)
        torch.cuda.synchronize()
        rec = oracle_desc(w.buf, offs, lens)
        compare(res, rec)
        c = res.counter_dict()
        assert c["l4_csum_bad"] == w.expect["l4_bad"] and c["ip_csum_bad"] == w.expect["ip_bad"]
