#!/usr/bin/env python3
"""Kernel tuning harness: times pnetgpu_rx_process per workload under several
env settings (e.g. PNETGPU_BLOCKS_PER_CU) in ONE process, interleaved rounds.

  python tools/kbench.py --workloads udp64,tcp1500 --env PNETGPU_BLOCKS_PER_CU=1,2,3,4,6,8
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libpnet_amd as lp  # noqa: E402
import bench  # noqa: E402
bench.load_library()
from bench import Shard, HBM_PEAK_GBS, WORKLOADS  # noqa: E402

EXTRA = {"imix": 1 << 22, "udp6_jumbo": 1 << 17}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="udp64,tcp1500")
    ap.add_argument("--env", default="")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tx", action="store_true", help="time tx_fill_checksums instead of rx_process")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    # --env KEY=v1,v2 or --env "K1=a+K2=b,K1=c+K2=d" (each comma-separated item one setting)
    if a.env and "+" not in a.env and a.env.count("=") == 1:
        key, vs = a.env.split("=")
        configs = [(f"{key}={v}", {key: v}) for v in vs.split(",")]
    elif a.env:
        configs = [(item, dict(kv.split("=") for kv in item.split("+"))) for item in a.env.split(",")]
    else:
        configs = [("", {})]
    vals = [c[0] for c in configs]
    envs = dict(configs)
    s = torch.cuda.Stream()
    for name in a.workloads.split(","):
        n = WORKLOADS[name]["n"] if name in WORKLOADS else EXTRA[name]
        sh = Shard(name, n, 1, dev)
        if a.tx:
            st = lp.RxResult(sh.n, dev, ("status",), counters=False)

            def tx_step(stream, sh=sh, st=st):
                lp.tx_fill_checksums(sh.data, stride=sh.w.stride, frame_len=sh.w.frame_len, n_frames=sh.n, out=st,
                                     stream=stream)
            sh.step = tx_step
        times = {v: [] for v in vals}
        for _ in range(a.rounds):
            for v in vals:
                lp.engine.apply_tuning_env(envs[v], dev)   # the context reads no env per call
                for _ in range(2):
                    sh.step(s)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
                for e0, e1 in evs:
                    e0.record(s)
                    sh.step(s)
                    e1.record(s)
                s.synchronize()
                times[v] += [e0.elapsed_time(e1) for e0, e1 in evs]
        for v in vals:
            t = np.array(times[v])
            med = float(np.median(t))
            print(f"{name:10s} {v}: median {med*1e3:8.1f} us  min {t.min()*1e3:8.1f} us  "
                  f"alg {sh.alg_bytes/med/1e6:7.0f} GB/s ({sh.alg_bytes/med/1e6/HBM_PEAK_GBS:.1%})  "
                  f"{sh.n/med/1e3:9.0f} Mpkts/s", flush=True)
        del sh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
