#!/usr/bin/env python3
"""Wave-level timing probe of the receive kernels: how evenly the persistent
waves of one launch finish (the kernel ends with its last wave).

Needs the variant library built with the probe:
  make -C libpnet_amd variant V=wt DEFS=-DPNET_WAVE_TIMES
  PNETGPU_LIB=$PWD/libpnet_amd/build/libpnetgpu_wt.so python tools/wave_times.py --workloads udp64,imix

Per launch it prints the span (first wave start -> last wave end), the end-time
percentiles, the per-XCD medians and maxima, and for descriptor batches the
correlation of a wave's duration with the frame bytes of its runs.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libpnet_amd as lp  # noqa: E402
import bench  # noqa: E402
bench.load_library()
from bench import Shard, WORKLOADS  # noqa: E402
from libpnet_amd import _lib  # noqa: E402

EXTRA = {"imix": 1 << 22, "udp6_jumbo": 1 << 17}
SLOTS, WORDS = 16384, 13
TICK_US = 0.01   # wall_clock64: 100 MHz


def read_times():
    buf = np.zeros(SLOTS * WORDS, dtype=np.uint64)
    rc = _lib._lib.pnetgpu_probe_wave_times(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.size), 0)
    assert rc == 0, "probe copy failed"
    return buf.reshape(SLOTS, WORDS)


def clear_times():
    assert _lib._lib.pnetgpu_probe_wave_times(None, ctypes.c_size_t(0), 1) == 0


def wave_bytes(sh, nwaves):
    """Frame bytes each wave's runs cover (grid-stride run order), descriptor batches."""
    lens = sh.w.lengths.astype(np.int64) if not sh.w.stride else np.full(sh.n, sh.w.frame_len, np.int64)
    nruns = (sh.n + 63) // 64
    pad = np.zeros(nruns * 64, np.int64)
    pad[:sh.n] = lens
    per_run = pad.reshape(nruns, 64).sum(1)
    out = np.zeros(nwaves, np.int64)
    np.add.at(out, np.arange(nruns) % nwaves, per_run)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="udp64,tcp1500,imix")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--save", default="", help="directory: raw per-wave records of each last rep (.npy)")
    ap.add_argument("--tag", default="")
    ap.add_argument("--env", default="", help="KEY=v1,v2: rerun every workload per value (e.g. PNETGPU_STATIC_PCT)")
    a = ap.parse_args()
    key, vals = (a.env.split("=") + [""])[:2] if a.env else ("", "")
    vals = vals.split(",") if vals else [None]
    f = _lib._lib.pnetgpu_probe_wave_times
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    for name in a.workloads.split(","):
        n = WORKLOADS[name]["n"] if name in WORKLOADS else EXTRA[name]
        sh = Shard(name, n, 1, dev)
        for _ in range(3):
            sh.step(s)
        s.synchronize()
        for v, rep in [(v, r) for v in vals for r in range(a.reps)]:
            if key:
                lp.engine.apply_tuning_env({key: v}, dev)
                if rep == 0:
                    print(f"-- {key}={v}", flush=True)
                    sh.step(s)
            clear_times()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            sh.step(s)
            e1.record(s)
            s.synchronize()
            ev_us = e0.elapsed_time(e1) * 1e3
            t = read_times()
            if a.save and rep == a.reps - 1:
                os.makedirs(a.save, exist_ok=True)
                np.save(os.path.join(a.save, f"wt_{name}_{a.tag}{v or ''}.npy"), t)
            live = t[:, 1] != 0
            t = t[live]
            nw = int(live.sum())
            t0 = t[:, 0].astype(np.int64)
            t1 = t[:, 1].astype(np.int64)
            base = t0.min()
            end = (t1 - base) * TICK_US
            start = (t0 - base) * TICK_US
            dur = end - start
            span = end.max()
            xcc = (t[:, 2] >> np.uint64(32)).astype(np.int64)
            runs = t[:, 3].astype(np.int64)
            pct = np.percentile(end, [1, 10, 50, 90, 99])
            print(f"{name:10s} rep {rep}: event {ev_us:7.1f} us, span {span:7.1f} us, waves {nw}, runs/wave "
                  f"{runs.min()}-{runs.max()}, start spread {start.max():5.1f} us; end p1 {pct[0]:6.1f} p10 "
                  f"{pct[1]:6.1f} p50 {pct[2]:6.1f} p90 {pct[3]:6.1f} p99 {pct[4]:6.1f} max {span:6.1f}; "
                  f"tail (max-p50)/span {(span - pct[2]) / span:5.1%}, mean busy/span {dur.mean() / span:5.1%}",
                  flush=True)
            if rep == a.reps - 1:
                print(f"{'':10s} runs total {runs.sum()} (batch {(sh.n + 63) // 64})", flush=True)
                clk = t[:, 9].astype(np.float64)
                if clk.max() > 0:
                    mhz = clk / np.maximum(dur, 1e-9)            # s_memtime ticks per us
                    ph = t[:, 4:8].astype(np.float64) / mhz[:, None] / np.maximum(runs, 1)[:, None]
                    names = ("window/loads", "tail", "parse", "stores")
                    print(f"{'':10s} per run (us, mean over waves; s_memtime {np.median(mhz):.0f} MHz): " +
                          "  ".join(f"{nm} {ph[:, i].mean():.2f}" for i, nm in enumerate(names)) +
                          f"  total {ph.sum(1).mean():.2f} ({dur.mean() / runs.mean():.2f} wall)", flush=True)
                tu, tsl, tid = (int(t[:, k].astype(np.int64).sum()) for k in (10, 11, 12))
                if tsl:
                    print(f"{'':10s} tail makespan: group-rounds issued {tu}, slots {tsl} (used {tu / tsl:.1%}); "
                          f"a perfect split needs {tid} slots ({tid / tsl:.1%} of the rounds), "
                          f"{tu / runs.sum():.1f} group-rounds per run", flush=True)
                per = []
                for x in range(8):
                    m = xcc == x
                    if m.any():
                        per.append(f"x{x}:{np.median(end[m]):.0f}/{end[m].max():.0f}({int(m.sum())})")
                print(f"{'':10s} per-XCD end median/max (waves): " + " ".join(per), flush=True)
                wid = np.nonzero(live)[0]
                if len(wid) == nw and wid.max() == nw - 1:
                    wb = wave_bytes(sh, nw)
                    c = np.corrcoef(wb, dur)[0, 1] if wb.std() > 0 else float("nan")
                    print(f"{'':10s} wave bytes: min {wb.min()/1e3:.0f} KB max {wb.max()/1e3:.0f} KB "
                          f"(max/mean {wb.max()/wb.mean():.3f}, std/mean {wb.std()/wb.mean():.3f}); "
                          f"corr(bytes, duration) {c:.2f}; duration max/mean {dur.max()/dur.mean():.3f}", flush=True)
        del sh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
