#!/usr/bin/env python3
"""Does the host pack's rate into pinned memory depend on which NUMA node the
pool's threads run on? The GPU's NUMA node (sysfs), then one child process per
CPU set — each node's CPUs within the allowed mask, and the whole mask — each
timing pnetgpu_batch_pack (2^20 64-B frames) into torch-pinned and pageable
destinations and the copying ring's push_many inside a running ring.

    python tools/probes/numa_probe.py [--seconds 1]
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def parse_cpulist(text):
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def nodes():
    out = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        with open(os.path.join(d, "cpulist")) as fh:
            out[int(d.rsplit("node", 1)[1])] = parse_cpulist(fh.read())
    return out


def child(seconds):
    import numpy as np
    import torch
    import bench
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", 1 << 22, 1000, dev)
    offs, lens = bench._ring_source(sh)
    src = sh.w.buf
    n = 1 << 20
    do, dl = np.zeros(n, np.uint64), np.zeros(n, np.uint32)
    out = {"cpus": len(os.sched_getaffinity(0)), "host_threads": lp.host_threads()}
    for name, dst in (("pinned", torch.empty(64 << 20, dtype=torch.uint8).pin_memory().numpy()),
                      ("pageable", np.ones(64 << 20, np.uint8))):
        lp.batch_pack(src, offs[:n], lens[:n], dst, do, dl, check_bounds=False)
        frames = i = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            k, _ = lp.batch_pack(src, offs[i:i + n], lens[i:i + n], dst, do, dl, check_bounds=False)
            frames += k
            i = (i + k) % (len(offs) - n + 1)
        out[f"pack_{name}_gb_s"] = round(frames * 64 / (time.perf_counter() - t0) / 1e9, 1)
    r = bench.e2e_ring_rate(sh, seconds=2 * seconds)
    out["ring_link_gb_s"] = r["link_gb_s"]
    out["ring_push_gb_s"] = r["stages"].get("push_gb_s")
    z = bench.e2e_zero_copy_rate(sh, seconds=2 * seconds)
    out["zero_copy_link_gb_s"] = z["link_gb_s"]
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a.seconds)
    allowed = os.sched_getaffinity(0)
    gpu_node = None
    for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            with open(p) as fh:
                v = int(fh.read())
            with open(os.path.join(os.path.dirname(p), "vendor")) as fh:
                if fh.read().strip() == "0x1002":
                    gpu_node = v
                    break
        except (OSError, ValueError):
            continue
    nd = nodes()
    print(json.dumps({"gpu_numa_node": gpu_node, "nodes": {k: len(v & allowed) for k, v in nd.items()},
                      "allowed": len(allowed)}), flush=True)
    sets = [(f"node{k}", sorted(v & allowed)) for k, v in nd.items() if v & allowed] + [("all", sorted(allowed))]
    for rnd in range(2):
        for name, cpus in (sets if rnd == 0 else list(reversed(sets))):
            code = (f"import os, sys; os.sched_setaffinity(0, {cpus!r}); sys.argv = [{__file__!r}, '--child', "
                    f"'--seconds', '{a.seconds}']; sys.path.insert(0, {ROOT!r}); "
                    f"import runpy; runpy.run_path({__file__!r}, run_name='__main__')")
            p = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=300)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            print(json.dumps({"round": rnd, "cpu_set": name, "rc": p.returncode,
                              **(json.loads(line[-1]) if line else {"err": p.stderr[-500:]})}), flush=True)
            if p.returncode:
                return p.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
