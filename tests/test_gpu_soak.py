"""A randomized soak of the receive and TX entry points against the oracle: many
small batches, each with a random batch form (fixed stride at a random
alignment — which is what routes 64-B frames to rx_small_kernel —, full or
compact descriptors), a random frame mix (valid / corrupted / truncated /
padded, VLAN and IPv6 extension frames when the flags ask for them), random
dispatch flags, a random frame-size hint (which picks the mixed, MTU or jumbo
tail shape for descriptor batches and must be ignored in stride mode), a
random subset of the result columns (which picks the plain, FIELDS and EXT
instantiations and the small kernel's linear-slot paths), a misaligned data
pointer, and receive or TX. Every column, the counters and
(TX) the patched bytes must equal the oracle's."""
import numpy as np
import pytest
import torch

import libpnet_amd as lp
from libpnet_amd.engine import ALL_COLUMNS, RX_IPV6_EXT, RX_VLAN
from oracle import coracle
from tests import framegen
from tests.test_gpu_parity import compare, oracle_counters, to_dev

pytestmark = pytest.mark.gpu

FLAG_SETS = (0, 0, 0, RX_VLAN, RX_IPV6_EXT, RX_VLAN | RX_IPV6_EXT)


def _frames(rng, n, flags, fixed_len):
    if fixed_len:
        kinds = ("udp", "tcp", "icmp", "udp6", "tcp6", "icmp6")
        out = []
        for _ in range(n):
            k = kinds[int(rng.integers(0, len(kinds)))]
            hdr = 14 + (40 if k.endswith("6") else 20)
            f = bytearray(framegen.build_frame(rng, k, max(0, fixed_len - hdr)))[:fixed_len]
            f += bytes(fixed_len - len(f))
            if rng.random() < 0.1:                      # a flipped byte: checksum mismatch
                f[int(rng.integers(0, fixed_len))] ^= 0x5A
            out.append(bytes(f))
        return out
    fr = framegen.random_frames(rng, n, max_len=int(rng.choice([100, 700, 1600, 9100])))
    if flags:
        fr += framegen.extension_frames(rng)[: max(1, n // 4)]
    return fr


@pytest.mark.parametrize("seed", range(6))
def test_random_batches_soak(seed):
    rng = np.random.default_rng(7000 + seed)
    for it in range(12):
        flags = int(FLAG_SETS[int(rng.integers(0, len(FLAG_SETS)))])
        form = ("stride", "desc", "compact")[int(rng.integers(0, 3))]
        tx = bool(rng.random() < 0.3)
        ncols = int(rng.integers(1, len(ALL_COLUMNS) + 1))
        cols = tuple(c for c in ALL_COLUMNS if c in set(rng.choice(ALL_COLUMNS, ncols, replace=False)))
        n = int(rng.integers(1, 900))
        mis = int(rng.integers(0, 16))
        what = (seed, it, form, flags, tx, cols)   # (the hint is drawn below)
        if form == "stride":
            flen = int(rng.choice([40, 54, 60, 64, 64, 64, 100, 576, 1500]))
            stride = flen + int(rng.choice([0, 0, 0, 4, 16, 64]))
            frames = _frames(rng, n, flags, flen)
            body = np.zeros(n * stride + 64, np.uint8)
            for i, f in enumerate(frames):
                body[i * stride:i * stride + flen] = np.frombuffer(f, np.uint8)
            host = np.concatenate([np.zeros(mis, np.uint8), body])
            full = to_dev(np.concatenate([np.zeros(16, np.uint8), host]))
            d = full[16 + mis:]
            kw = dict(stride=stride, frame_len=flen, n_frames=n)
            okw = dict(stride=stride, frame_len=flen)
            lens = np.full(n, flen, np.uint32)
            want_src = body
        else:
            frames = _frames(rng, n, flags, 0)
            n = len(frames)
            buf, offs, lens = framegen.pack(frames, gap=int(rng.integers(0, 20)), rng=rng)
            full = to_dev(np.concatenate([np.zeros(16 + mis, np.uint8), buf, np.zeros(32, np.uint8)]))
            d = full[16 + mis:16 + mis + buf.size]
            if form == "compact":
                kw = dict(offsets=to_dev(offs.astype(np.uint32).view(np.int32)),
                          lengths=to_dev(lens.astype(np.uint16).view(np.int16)))
                fl = flags | lp.DESC_COMPACT
            else:
                kw = dict(offsets=to_dev(offs.astype(np.int64)), lengths=to_dev(lens.astype(np.int32)))
                fl = flags
            okw = dict(offsets=offs, lengths=lens)
            want_src = buf
        hint = int(rng.choice([0, 0, lp.DESC_HINT_LARGE, lp.DESC_HINT_JUMBO]))
        call_flags = (fl if form != "stride" else flags) | hint
        if tx:
            want_buf, rec = coracle.tx_fill(want_src, n, flags=flags, **okw)
            res = lp.tx_fill_checksums(d, columns=cols, counters=True, flags=call_flags, **kw)
        else:
            rec = coracle.rx_batch(want_src, n, flags=flags, **okw)
            res = lp.rx_process(d, columns=cols, flags=call_flags, **kw)
        torch.cuda.synchronize()
        compare(res, rec)
        assert res.counter_dict() == oracle_counters(rec, lens), what
        if tx:
            got = d.cpu().numpy()
            assert np.array_equal(got[:want_buf.size], want_buf[:got.size]), what
