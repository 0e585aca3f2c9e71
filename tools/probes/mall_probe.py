#!/usr/bin/env python3
"""Does back-to-back replay of one resident batch gain from the 256 MiB
Infinity Cache? Times each workload replaying 1 batch vs rotating over 2 and 3
distinct batches of the same shape (reuse distance x2, x3)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
bench.load_library()
from bench import Shard, WORKLOADS, HBM_PEAK_GBS  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    for name in (sys.argv[1] if len(sys.argv) > 1 else "udp64,tcp1500,imix,udp6_jumbo").split(","):
        shards = [Shard(name, WORKLOADS[name]["n"], seed, dev) for seed in (1, 2, 3)]
        for k in (1, 2, 3, 1):
            for i in range(6):
                shards[i % k].step(s)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(24)]
            for i, (e0, e1) in enumerate(evs):
                e0.record(s)
                shards[i % k].step(s)
                e1.record(s)
            s.synchronize()
            t = np.array([e0.elapsed_time(e1) for e0, e1 in evs])
            med = float(np.median(t))
            print(f"{name:10s} rotate {k}: median {med*1e3:7.1f} us  alg {shards[0].alg_bytes/med/1e6:6.0f} GB/s "
                  f"({shards[0].alg_bytes/med/1e6/HBM_PEAK_GBS:.1%})", flush=True)
        del shards
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
