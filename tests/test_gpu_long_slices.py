"""GPU parity of the batched util::* checksums on slices long enough for the
reference's u32 sums to wrap (util.rs:103-114,139-149,158-181: `sum += ...` in a
release build wraps modulo 2^32; the oracle restates that). Below kExactMax =
65536 bytes (slice + extra) nothing can wrap; above it the slice kernels also
sum the plain bytes T and take the word sum as S or 257 T - S, exact modulo
2^32 (rx_slices.h, group_range_sum_t). Slices of 0xFF bytes (every word 0xFFFF: the most
wraps), random bytes, every alignment, skipped words anywhere (also inside a
slice's last granule and its odd trailing byte), mixed with short slices in one
batch, through each descriptor kernel (the slice_kernel tuning) and the strided
form, util::checksum, ipv4 / ipv6_checksum and their *_adv forms."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from oracle import coracle
from tests.test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu

LONG = [65537, 65538, 131071, 131072, 200001, (1 << 20) + 3, 5 << 20]


def _batch(rng, fill):
    """A buffer and slices: the long ones at offsets 0..15, short ones between."""
    size = (6 << 20) + 64
    buf = np.full(size, 0xFF, np.uint8) if fill == "ff" else rng.integers(0, 256, size, dtype=np.uint8)
    offs, lens, skips = [], [], []
    for k, ln in enumerate(LONG):
        o = int(rng.integers(0, size - ln - 16)) & ~15
        offs.append(o + k % 16)
        lens.append(ln)
        skips.append(int(rng.choice([0, 5, ln // 2, (ln - 1) // 2, ln, 1 << 30])))
    for _ in range(200):                       # short slices in the same runs / units
        ln = int(rng.integers(0, 3000))
        offs.append(int(rng.integers(0, size - ln)))
        lens.append(ln)
        skips.append(int(rng.integers(0, 40)))
    order = rng.permutation(len(offs))
    return (buf, np.array(offs, np.int64)[order], np.array(lens, np.int32)[order],
            np.array(skips, np.int32)[order])


@pytest.mark.parametrize("fill", ["ff", "random"])
@pytest.mark.parametrize("kernel", [None, "run", "group", "tiny"])
def test_long_checksum_slices(fill, kernel, tune):
    rng = np.random.default_rng(41 + len(fill))
    buf, offs, lens, skips = _batch(rng, fill)
    tune("slice_kernel", None if kernel is None else {"run": 1, "group": 2, "tiny": 3}[kernel])
    want = coracle.checksum_slices(buf, offs.astype(np.uint64), lens.astype(np.uint32), skips.astype(np.uint32))
    got = lp.checksum_slices(to_dev(buf), to_dev(offs), to_dev(lens), to_dev(skips))
    torch.cuda.synchronize()
    got = got.cpu().numpy().view(np.uint16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(lens[i]), int(offs[i]) & 15, int(skips[i]), hex(got[i]), hex(want[i])) for i in bad[:5]]


@pytest.mark.parametrize("version", [4, 6])
@pytest.mark.parametrize("kernel", [None, "run", "group"])
def test_long_pseudo_header_slices(version, kernel, tune):
    rng = np.random.default_rng(43 + version)
    buf, offs, lens, skips = _batch(rng, "ff")
    n = len(offs)
    alen = 4 if version == 4 else 16
    addrs = rng.integers(0, 256, (n, 2 * alen), dtype=np.uint8)
    addrs[: n // 2] = 0xFF                               # the largest pseudo-header sums
    protos = rng.integers(0, 256, n, dtype=np.uint8)
    # extra slices (the *_adv form): long ones, odd lengths, empty
    eoffs = rng.integers(0, buf.size - 70000, n).astype(np.int64)
    elens = rng.choice([0, 1, 7, 65535, 65537, 70000 - 1], n).astype(np.int32)
    tune("slice_kernel", None if kernel is None else {"run": 1, "group": 2}[kernel])
    fn = coracle.ipv4_checksum if version == 4 else coracle.ipv6_checksum
    want = np.array([fn(buf[o:o + ln], sk, b"", a[:alen].tobytes(), a[alen:].tobytes(), int(p))
                     for o, ln, sk, a, p in zip(offs, lens, skips, addrs, protos)], np.uint16)
    slices = lp.ipv4_checksum_slices if version == 4 else lp.ipv6_checksum_slices
    got = slices(to_dev(buf), to_dev(offs), to_dev(lens), to_dev(skips), to_dev(addrs), to_dev(protos))
    want_adv = np.array([fn(buf[o:o + ln], sk, buf[eo:eo + el].tobytes(), a[:alen].tobytes(), a[alen:].tobytes(),
                            int(p))
                         for o, ln, sk, eo, el, a, p in zip(offs, lens, skips, eoffs, elens, addrs, protos)], np.uint16)
    got_adv = lp.checksum_adv_slices(version, to_dev(buf), to_dev(offs), to_dev(lens), to_dev(skips), to_dev(eoffs),
                                     to_dev(elens), to_dev(addrs), to_dev(protos))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint16), want)
    assert np.array_equal(got_adv.cpu().numpy().view(np.uint16), want_adv)


@pytest.mark.parametrize("slice_len", [65537, 131072, 1 << 20])
def test_long_strided_slices(slice_len):
    """Uniform long slices (pnetgpu_checksum_slices_strided; the group kernel),
    overlapping (stride < slice_len) and repeated (stride 0)."""
    buf = np.full((4 << 20) + 64, 0xFF, np.uint8)
    buf[::977] = 0x12
    for stride, n in ((slice_len // 3 + 1, 6), (0, 3), (slice_len + 5, 2)):
        if (n - 1) * stride + slice_len > buf.size:
            n = max(1, (buf.size - slice_len) // max(stride, 1) + 1)
        want = np.array([coracle.checksum(buf[i * stride:i * stride + slice_len], 7) for i in range(n)], np.uint16)
        got = lp.checksum_slices_strided(to_dev(buf), n, stride, slice_len, 7)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint16), want), (stride, n)


@pytest.mark.parametrize("version", [4, 6])
def test_long_extra_with_empty_data_in_a_dense_run(version, tune):
    """An *_adv slice whose data is empty and whose extra slice is past
    kExactMax, in a run of small packed slices (slice_run_kernel's dense LDS
    stage would otherwise take the run)."""
    rng = np.random.default_rng(47 + version)
    buf = rng.integers(0, 256, 300000, dtype=np.uint8)
    buf[100000:] = 0xFF
    lens = rng.integers(30, 45, 64).astype(np.int32)
    offs = np.concatenate([[16], 16 + np.cumsum(lens[:-1])]).astype(np.int64)
    lens[17] = 0                                      # the empty data slice
    skips = np.full(64, 3, np.int32)
    eoffs = np.full(64, 8, np.int64)
    elens = np.full(64, 10, np.int32)
    eoffs[17], elens[17] = 100001, 150001             # its long extra slice
    alen = 4 if version == 4 else 16
    addrs = np.full((64, 2 * alen), 0xFF, np.uint8)
    protos = np.full(64, 17, np.uint8)
    tune("slice_kernel", "run")
    fn = coracle.ipv4_checksum if version == 4 else coracle.ipv6_checksum
    want = np.array([fn(buf[o:o + ln], sk, buf[eo:eo + el].tobytes(), a[:alen].tobytes(), a[alen:].tobytes(), int(p))
                     for o, ln, sk, eo, el, a, p in zip(offs, lens, skips, eoffs, elens, addrs, protos)], np.uint16)
    got = lp.checksum_adv_slices(version, to_dev(buf), to_dev(offs), to_dev(lens), to_dev(skips), to_dev(eoffs),
                                 to_dev(elens), to_dev(addrs), to_dev(protos))
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().view(np.uint16), want)
