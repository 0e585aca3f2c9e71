#!/usr/bin/env python3
"""Fixed cost per launch of the fixed-stride receive kernels: back-to-back
launches (one HIP event pair around 20 of them, as bench.py times) over the
first n frames of the same resident batch, n halved four times; a least-squares
line t(n) = t0 + n * t1 separates the per-launch cost t0 (dispatch, the last
waves' tail, the end-of-kernel cache write-back) from the per-frame cost.
Interleaved rounds, medians."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
bench.load_library()
import libpnet_amd as lp  # noqa: E402
from bench import Shard, WORKLOADS  # noqa: E402


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["udp64", "tcp1500"]
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    for name in names:
        sh = Shard(name, WORKLOADS[name]["n"], 1, dev)
        sizes = [sh.n >> k for k in range(5)]
        res = {n: lp.RxResult(n, dev, lp.IPV4_COLUMNS, counters=True) for n in sizes}
        times = {n: [] for n in sizes}
        for _ in range(5):
            for n in sizes:
                fn = (lambda st, n=n: lp.rx_process(sh.data, stride=sh.w.stride, frame_len=sh.w.frame_len,
                                                    n_frames=n, out=res[n], stream=st))
                times[n].append(bench.time_launches(fn, 20, 3, s) * 1e3)
        med = np.array([np.median(times[n]) for n in sizes])
        x = np.array(sizes, np.float64)
        t1, t0 = np.polyfit(x, med, 1)
        for n, t in zip(sizes, med):
            print(f"{name:8s} n {n:9d}: {t:8.1f} us per launch (fit {t0 + t1 * n:8.1f})", flush=True)
        print(f"{name:8s} fixed per launch {t0:6.1f} us = {t0 / med[0]:.1%} of the full batch; "
              f"{t1 * 1e3:.3f} ns per frame", flush=True)


if __name__ == "__main__":
    main()
