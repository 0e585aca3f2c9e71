#!/usr/bin/env python3
"""Does the zero-copy ring's rate depend on which hardware queues its two
streams land on? HIP spreads a process's streams over GPU_MAX_HW_QUEUES
hardware queues (4 on the GPU boxes); two streams sharing one queue run
every operation of both in one order, with no copy/copy-back overlap. One
child process per count of extra streams created (and kept) before the ring,
each timing bench.e2e_zero_copy_rate and bench.e2e_ring_rate.

    python tools/probes/hwq_probe.py [--extra 0,1,2,3,4,5] [--seconds 2]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def child(extra, seconds):
    import torch
    import bench
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", 1 << 22, 1000, dev)
    keep = [torch.cuda.Stream(dev) for _ in range(extra)]
    for s in keep:                                  # make sure each is really created on the device
        with torch.cuda.stream(s):
            torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    z = bench.e2e_zero_copy_rate(sh, seconds=seconds)
    r = bench.e2e_ring_rate(sh, seconds=seconds)
    print(json.dumps({"extra_streams": extra, "zero_copy": z["link_gb_s"], "ring": r["link_gb_s"],
                      "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--extra", default="0,1,2,3,4,5")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--child", type=int, default=-1)
    a = ap.parse_args()
    if a.child >= 0:
        return child(a.child, a.seconds)
    for e in [int(x) for x in a.extra.split(",")]:
        p = subprocess.run([sys.executable, "-u", __file__, "--child", str(e), "--seconds", str(a.seconds)],
                           capture_output=True, text=True, timeout=300)
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        print(lines[-1] if lines else json.dumps({"extra_streams": e, "rc": p.returncode, "err": p.stderr[-400:]}),
              flush=True)
        if p.returncode:
            return p.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
