#!/usr/bin/env python3
"""Descriptor batches (compact u32/u16 descriptors, as the ring and the
AF_PACKET path ship them) of different size mixes through each rx_kernel tail
shape — mixed (G=4, U=8, windows first, short runs), MTU (G=8, U=4, unified)
and jumbo (G=64, U=9) — forced with the rx_kind tuning. Interleaved rounds on
one box, kernel time per launch from one event pair around back-to-back
launches, records of every shape compared with the mixed shape's.

Batches (~1.2-1.6 GiB each): udp1500 frames packed; tcp1500 frames packed; a
1:1 mix of 64-B and 1500-B frames; 576-B frames (IMIX's middle class); IMIX;
cutL: the first L bytes of udp1500 frames packed (L = 768 ... 1280: where the
shapes cross); jumbo9000: 9000-B IPv6 frames packed; jmix: 64-B and 9000-B
frames at 7:1.

  python tools/probes/desc_shape_probe.py [--rounds 3] [--reps 10]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402

KINDS = {"mixed": 0, "mtu": 2, "jumbo": 3}


def packed(frames_buf, lens):
    """Frames given back to back: the buffer and compact descriptors."""
    offs = np.zeros(lens.size, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    return frames_buf, offs, lens


def build(name):
    if name in ("udp1500", "tcp1500"):
        n = 1 << 20
        w = lp.synth.make(name, n, seed=41, corrupt_ppm=10000)
        return packed(w.buf, np.full(n, 1500, np.uint32))
    if name == "imix":
        w = lp.synth.make("imix", 1 << 22, seed=41, corrupt_ppm=10000)
        return w.buf, w.offsets, w.lengths
    if name == "mix64_1500":
        n = 1 << 21                                   # 2^20 of each, interleaved 1:1
        a = lp.synth.make("udp64", n // 2, seed=42, corrupt_ppm=10000)
        b = lp.synth.make("udp1500", n // 2, seed=43, corrupt_ppm=10000)
        buf = np.zeros((n // 2) * (64 + 1500) + 64, np.uint8)
        pair = buf[: (n // 2) * 1564].reshape(n // 2, 1564)
        pair[:, :64] = a.buf[: (n // 2) * 64].reshape(-1, 64)
        pair[:, 64:] = b.buf[: (n // 2) * 1500].reshape(-1, 1500)
        lens = np.tile(np.array([64, 1500], np.uint32), n // 2)
        return packed(buf, lens)
    if name == "only576":
        w = lp.synth.make("imix", 1 << 23, seed=44, corrupt_ppm=10000)
        keep = np.nonzero(w.lengths == 576)[0][: 1 << 21]
        buf = np.zeros(keep.size * 576 + 64, np.uint8)
        frames = buf[: keep.size * 576].reshape(-1, 576)
        for k in range(0, keep.size, 4096):
            idx = keep[k:k + 4096]
            src = w.offsets[idx][:, None] + np.arange(576, dtype=np.uint64)[None, :]
            frames[k:k + idx.size] = w.buf[src.astype(np.int64)]
        return packed(buf, np.full(keep.size, 576, np.uint32))
    if name.startswith("cut"):                        # the first L bytes of udp1500 frames, packed
        L = int(name[3:])
        n = min(1 << 20, (1536 << 20) // L)
        w = lp.synth.make("udp1500", n, seed=45, corrupt_ppm=10000)
        buf = np.zeros(n * L + 64, np.uint8)
        buf[: n * L].reshape(n, L)[:] = w.buf[: n * 1500].reshape(n, 1500)[:, :L]
        return packed(buf, np.full(n, L, np.uint32))
    if name == "jumbo9000":
        n = 1 << 17
        w = lp.synth.make("udp6_jumbo", n, seed=46, corrupt_ppm=10000)
        return packed(w.buf, np.full(n, 9000, np.uint32))
    if name == "jmix":                                # 7:1 64-B and 9000-B frames
        k = 1 << 16
        a = lp.synth.make("udp64", 7 * k, seed=47, corrupt_ppm=10000)
        b = lp.synth.make("udp6_jumbo", k, seed=48, corrupt_ppm=10000)
        grp = 7 * 64 + 9000
        buf = np.zeros(k * grp + 64, np.uint8)
        g = buf[: k * grp].reshape(k, grp)
        g[:, :448] = a.buf[: 7 * k * 64].reshape(k, 448)
        g[:, 448:] = b.buf[: k * 9000].reshape(k, 9000)
        lens = np.tile(np.array([64] * 7 + [9000], np.uint32), k)
        return packed(buf, lens)
    raise KeyError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="udp1500,tcp1500,mix64_1500,only576,imix")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = lp.engine.context(0)
    s = torch.cuda.Stream()
    ok = True
    for name in a.batches.split(","):
        buf, offs, lens = build(name)
        n = lens.size
        d = torch.from_numpy(buf).to(dev)
        o = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).to(dev)
        ln = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev)
        alg = int(lens.sum()) + n * (26 + 6)
        res = {k: lp.RxResult(n, dev, lp.IPV4_COLUMNS, counters=True) for k in KINDS}
        times = {k: [] for k in KINDS}
        for rnd in range(a.rounds):
            for k, kind in KINDS.items():
                ctx.set_tuning("rx_kind", kind)
                with torch.cuda.stream(s):
                    for _ in range(2):
                        lp.rx_process(d, offsets=o, lengths=ln, out=res[k], stream=s, flags=lp.DESC_COMPACT)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(a.reps):
                        lp.rx_process(d, offsets=o, lengths=ln, out=res[k], stream=s, flags=lp.DESC_COMPACT)
                    e1.record(s)
                s.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.reps)
        ctx.set_tuning("rx_kind", None)
        recs = {k: r.numpy() for k, r in res.items()}
        same = all(np.array_equal(recs[k][c], recs["mixed"][c]) for k in KINDS for c in lp.IPV4_COLUMNS)
        ok = ok and same
        line = "  ".join(f"{k} {min(t) * 1e3:6.1f}-{max(t) * 1e3:6.1f} us ({alg / min(t) / 1e9 / 8:.3f})"
                         for k, t in times.items())
        print(f"{name:11s} n={n:8d} avg {int(lens.sum()) / n:6.1f} B: {line}  records identical: {same}",
              flush=True)
        del d, o, ln, res
        torch.cuda.empty_cache()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
