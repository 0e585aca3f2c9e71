#!/usr/bin/env python3
"""The bench's producer lines (e2e_pcie, e2e_zero_copy, e2e_ring, pack only) for
one workload, once per host-pool size: each size runs in a child process with
PNETGPU_HOST_THREADS set (the pool is sized once per process). One JSON line per
size on stdout.

    python tools/e2e_probe.py --workload udp64 --threads 8,12,16 [--seconds 2]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(args):
    import torch
    import bench
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    n = int(bench.WORKLOADS[args.workload]["n"] * args.scale)
    sh = bench.Shard(args.workload, n, 1000, dev)
    out = {"workload": args.workload, "host_threads": lp.host_threads(),
           "env": os.environ.get("PNETGPU_HOST_THREADS")}
    out["pack_only"] = bench.pack_rate(sh)
    out["e2e_pcie"] = bench.e2e_rate(sh, dev)
    out["e2e_zero_copy"] = bench.e2e_zero_copy_rate(sh, seconds=args.seconds)
    out["e2e_ring"] = bench.e2e_ring_rate(sh, seconds=args.seconds)
    for v in out.values():
        if isinstance(v, dict):
            v.pop("note", None)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="udp64")
    ap.add_argument("--threads", default="")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--scale", type=float, default=0.25)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    for t in [x for x in args.threads.split(",") if x] or [None]:
        env = dict(os.environ)
        env.pop("PNETGPU_HOST_THREADS", None)
        if t:
            env["PNETGPU_HOST_THREADS"] = t
        rc = subprocess.run([sys.executable, "-u", __file__, "--child", "--workload", args.workload, "--seconds",
                             str(args.seconds), "--scale", str(args.scale)], env=env, timeout=300).returncode
        if rc:
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
