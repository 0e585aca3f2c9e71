#!/usr/bin/env python3
"""Does the zero-copy ring's rate depend on which NUMA node holds the frames it
DMAs, and on its page size? The same 2^22 64-B frames copied into anonymous
memory bound (mbind, MPOL_BIND) to each NUMA node in turn, with 4-KiB or
transparent 2-MiB pages, and the bench's own numpy source, page-locked (pnetgpu_host_register) and
shipped by the zero-copy ring (bench.e2e_zero_copy_rate's loop); the GPU's
node from sysfs. One process, interleaved rounds.

    python tools/probes/numa_zc_probe.py [--rounds 2] [--seconds 2]
"""
import argparse
import ctypes
import glob
import json
import mmap
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

SYS_MBIND = 237          # x86_64
MPOL_BIND = 2


def node_buffer(nbytes, node, thp=False):
    """Anonymous memory whose pages come from NUMA node `node` only (2-MiB
    transparent huge pages when thp)."""
    mm = mmap.mmap(-1, nbytes, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if thp:
        mm.madvise(mmap.MADV_HUGEPAGE)
    arr = np.frombuffer(mm, dtype=np.uint8)
    libc = ctypes.CDLL(None, use_errno=True)
    mask = ctypes.c_ulong(1 << node)
    rc = libc.syscall(SYS_MBIND, ctypes.c_void_p(arr.ctypes.data), ctypes.c_ulong(nbytes), MPOL_BIND,
                      ctypes.byref(mask), ctypes.c_ulong(64), 0)
    if rc != 0:
        raise OSError(ctypes.get_errno(), "mbind")
    return mm, arr


def gpu_node():
    for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            with open(os.path.join(os.path.dirname(p), "vendor")) as fh:
                if fh.read().strip() == "0x1002":
                    with open(p) as fh2:
                        return int(fh2.read())
        except (OSError, ValueError):
            continue
    return None


def zc_rate(lp, buf, offs, lens, seconds):
    reg = lp.HostRegistration(buf)
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=False, stage_times=True)
    frames = 0
    try:
        bench._ring_warm(ring, lambda: ring.feed_region(buf, offs, lens))
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for b in ring.feed_region(buf, offs, lens):
                frames += b.n
                del b
        for b in ring.drain():
            frames += b.n
        el = time.perf_counter() - t0
        st = ring.stats()
    finally:
        ring.close()
        reg.close()
    up = (st["bytes"] + st["desc_bytes"]) / max(st["frames"], 1)
    return {"link_gb_s": round(frames * (up + 26) / el / 1e9, 2),
            "h2d_gb_s": round(st["bytes"] / (st["h2d_ms"] / 1e3) / 1e9, 2) if st["h2d_ms"] else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", 1 << 22, 1000, dev)
    offs, lens = bench._ring_source(sh)
    span = int(offs[-1] + lens[-1])
    nodes = sorted(int(d.rsplit("node", 1)[1]) for d in glob.glob("/sys/devices/system/node/node[0-9]*"))
    bufs = {}
    for nd in nodes:
        for thp in (False, True):
            mm, arr = node_buffer(span, nd, thp)
            np.copyto(arr, sh.w.buf[:span])             # pages fault in on node nd
            bufs[f"node{nd}" + ("_thp" if thp else "")] = (mm, arr)
    bufs["numpy_buffer"] = (None, sh.w.buf[:span])      # the bench's source, as allocated
    print(json.dumps({"gpu_numa_node": gpu_node(), "nodes": nodes}), flush=True)
    out = {}
    for r in range(a.rounds):
        for k in (list(bufs) if r % 2 == 0 else list(reversed(bufs))):
            out.setdefault(k, []).append(zc_rate(lp, bufs[k][1], offs, lens, a.seconds))
            print(json.dumps({"round": r, "frames_on": k, **out[k][-1]}), flush=True)
    print(json.dumps({"summary": {k: [x["link_gb_s"] for x in v] for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
