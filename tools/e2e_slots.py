#!/usr/bin/env python3
"""PCIe-inclusive producer rates against the ring's slot count, one process,
same box: e2e_pcie (the plain two-stream pipeline) beside e2e_zero_copy and
e2e_ring at each slot count.

  python tools/e2e_slots.py --workload udp64 --slots 3,4,6,8
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="udp64")
    ap.add_argument("--slots", default="3,4,6,8")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--repeat", type=int, default=1, help="interleaved rounds (pcie, then every slot count)")
    a = ap.parse_args()
    bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard(a.workload, bench.WORKLOADS[a.workload]["n"], 1000, dev)
    out = {"workload": a.workload, "rounds": []}
    for r in range(a.repeat):
        rnd = {"e2e_pcie": bench.e2e_rate(sh, dev)}
        print(r, "pcie", rnd["e2e_pcie"]["link_gb_s"], file=sys.stderr, flush=True)
        for k in (int(x) for x in a.slots.split(",")):
            rnd[f"slots{k}"] = {"zero_copy": bench.e2e_zero_copy_rate(sh, a.seconds, slots=k),
                                "ring": bench.e2e_ring_rate(sh, a.seconds, slots=k)}
            print(r, k, rnd[f"slots{k}"]["zero_copy"]["link_gb_s"], rnd[f"slots{k}"]["ring"]["link_gb_s"],
                  file=sys.stderr, flush=True)
        out["rounds"].append(rnd)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
