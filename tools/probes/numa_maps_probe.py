#!/usr/bin/env python3
"""Which NUMA node holds the ring's pinned slots, torch's pinned memory and a
numpy batch? Pages per node from /proc/self/numa_maps for the mappings that
contain each buffer, and the GPU's node from sysfs.

    python tools/probes/numa_maps_probe.py
"""
import glob
import json
import os
import re
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def node_pages(addr):
    """{node: pages} of the numa_maps entry whose mapping starts at or before addr (the closest)."""
    best, best_start = None, -1
    with open("/proc/self/numa_maps") as fh:
        for ln in fh:
            start = int(ln.split()[0], 16)
            if best_start < start <= addr:
                best, best_start = ln, start
    if best is None:
        return {}
    return {"policy": best.split()[1], **{k: int(v) for k, v in re.findall(r"\b(N\d+)=(\d+)", best)}}


def main():
    lp = bench.load_library()
    torch.cuda.init()
    gpu = None
    for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
        with open(os.path.join(os.path.dirname(p), "vendor")) as fh:
            if fh.read().strip() == "0x1002":
                with open(p) as fh2:
                    gpu = int(fh2.read())
                break
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", 1 << 22, 1000, dev)
    offs, lens = bench._ring_source(sh)
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=False)
    slots = []
    for b in list(ring.feed_many(sh.w.buf, offs, lens)) + list(ring.drain()):
        slots.append(int(b._ptr[2]))
    pinned = torch.empty(64 << 20, dtype=torch.uint8).pin_memory()
    out = {"gpu_numa_node": gpu,
           "ring_slots": [node_pages(p) for p in sorted(set(slots))],
           "torch_pinned": node_pages(pinned.data_ptr()),
           "numpy_batch": node_pages(sh.w.buf.ctypes.data)}
    ring.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
