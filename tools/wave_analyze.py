#!/usr/bin/env python3
"""Offline analysis of tools/wave_times.py --save records: which hardware
position explains a wave's duration (wave slot on its SIMD, SIMD, CU, XCD,
dispatch order).  usage: python tools/wave_analyze.py gpurun_out/wt2/wt_udp64_s.npy ...
"""
import sys

import numpy as np

TICK_US = 0.01


def decode(t):
    live = t[:, 1] != 0
    wid = np.nonzero(live)[0]
    t = t[live]
    t0 = t[:, 0].astype(np.int64)
    t1 = t[:, 1].astype(np.int64)
    hw = (t[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    return {
        "wid": wid, "start": (t0 - t0.min()) * TICK_US, "end": (t1 - t0.min()) * TICK_US,
        "dur": (t1 - t0) * TICK_US, "xcc": (t[:, 2] >> np.uint64(32)).astype(np.int64),
        "slot": hw & 15, "simd": (hw >> 4) & 3, "cu": (hw >> 8) & 15, "sh": (hw >> 12) & 1,
        "se": (hw >> 13) & 7, "runs": t[:, 3].astype(np.int64),
    }


def by(d, key, vals):
    out = []
    for k in np.unique(key):
        m = key == k
        out.append((k, m.sum(), vals[m].mean(), vals[m].min(), vals[m].max()))
    return out


def report(path):
    d = decode(np.load(path)[:, :4] if np.load(path).shape[1] > 4 else np.load(path))
    dur = d["dur"]
    print(f"== {path}: {len(dur)} waves, duration mean {dur.mean():.1f} us, min {dur.min():.1f}, max {dur.max():.1f}")
    for name, key in [("wave slot", d["slot"]), ("simd", d["simd"]), ("xcc", d["xcc"]),
                      ("wave in block", d["wid"] % 4), ("dispatch round", (d["wid"] // 4) // 256)]:
        rows = by(d, key, dur)
        print(f"  by {name}: " + "  ".join(f"{k}:{m:.1f}[{lo:.0f}-{hi:.0f}](n={n})" for k, n, m, lo, hi in rows))
    cu = d["xcc"] * 64 + d["se"] * 32 + d["sh"] * 16 + d["cu"]
    rows = by(d, cu, dur)
    means = np.array([r[2] for r in rows])
    print(f"  per-CU mean duration over {len(rows)} CUs: min {means.min():.1f} p10 {np.percentile(means, 10):.1f} "
          f"p50 {np.median(means):.1f} p90 {np.percentile(means, 90):.1f} max {means.max():.1f}")
    # within-CU spread vs between-CU spread
    within = np.array([dur[cu == k].std() for k in np.unique(cu)])
    print(f"  std of duration: total {dur.std():.2f}, between CUs {means.std():.2f}, mean within-CU {within.mean():.2f}")
    # wave slot x SIMD table
    slot_rank = np.zeros_like(dur)
    for k in np.unique(cu):
        for sd in range(4):
            m = (cu == k) & (d["simd"] == sd)
            order = np.argsort(np.argsort(d["start"][m]))
            slot_rank[m] = order
    rows = by(d, slot_rank.astype(int), dur)
    print("  by start order on its SIMD: " + "  ".join(f"{k}:{m:.1f}(n={n})" for k, n, m, lo, hi in rows))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        report(p)
