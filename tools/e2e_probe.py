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


def cpu_stat():
    """The cgroup's CPU accounting (v2 cpu.stat, else v1): usage and throttling."""
    for path in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            with open(path) as fh:
                return {k: int(v) for k, v in (ln.split() for ln in fh if len(ln.split()) == 2)}
        except (OSError, ValueError):
            continue
    return {}


def timed(fn):
    """fn() with the cgroup's CPU usage and throttling over its run."""
    a = cpu_stat()
    out = fn()
    b = cpu_stat()
    if isinstance(out, dict) and a:
        out["cgroup"] = {k: b.get(k, 0) - a.get(k, 0) for k in ("usage_usec", "nr_periods", "nr_throttled",
                                                               "throttled_usec", "throttled_time") if k in a}
    return out


def child(args):
    import torch
    import bench
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    n = int(bench.WORKLOADS[args.workload]["n"] * args.scale)
    sh = bench.Shard(args.workload, n, 1000, dev)
    out = {"workload": args.workload, "host_threads": lp.host_threads(),
           "env": os.environ.get("PNETGPU_HOST_THREADS")}
    out["pack_only"] = timed(lambda: bench.pack_rate(sh))
    out["e2e_pcie"] = timed(lambda: bench.e2e_rate(sh, dev))
    out["e2e_zero_copy"] = timed(lambda: bench.e2e_zero_copy_rate(sh, seconds=args.seconds))
    out["e2e_ring"] = timed(lambda: bench.e2e_ring_rate(sh, seconds=args.seconds))
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
