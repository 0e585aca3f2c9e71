#!/usr/bin/env python3
"""Where the pinned ring's PCIe-inclusive rate goes: the bench's e2e_pcie
(plain double-buffered pipeline) beside the zero-copy ring driven (a) through
Ring.feed_region (a Batch object with numpy views per waited batch, as the
bench does) and (b) through the C-ABI directly from a ctypes loop
(submit_region / wait / release, no per-batch Python objects), interleaved.

  python tools/probes/ring_probe.py [--slots 4] [--rounds 2] [--seconds 3]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def raw_zero_copy(lp, sh, seconds, slots):
    from libpnet_amd._lib import check, lib
    from libpnet_amd.ring import EBUSY, EEMPTY, RingBatch
    w = sh.w
    n = sh.n
    offs = np.arange(n, dtype=np.uint64) * np.uint64(w.stride)
    lens = np.full(n, w.frame_len, np.uint32)
    buf = w.buf[: n * w.stride]
    reg = lp.HostRegistration(buf)
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=False, columns=lp.IPV4_COLUMNS, slots=slots)
    rb = RingBatch()
    taken, bid = ctypes.c_uint64(), ctypes.c_uint64()
    frames = 0
    t0 = time.perf_counter()
    try:
        while time.perf_counter() - t0 < seconds:
            i = 0
            while i < n:
                rc = lib.pnetgpu_ring_submit_region(ring.h, ctypes.c_void_p(buf.ctypes.data),
                                                    ctypes.c_void_p(offs[i:].ctypes.data),
                                                    ctypes.c_void_p(lens[i:].ctypes.data), n - i, ctypes.byref(taken),
                                                    ctypes.byref(bid))
                if rc == 0:
                    i += taken.value
                    continue
                if rc != EBUSY:
                    check(rc, "submit_region")
                check(lib.pnetgpu_ring_wait(ring.h, ctypes.byref(rb)), "wait")
                frames += rb.n_frames
                check(lib.pnetgpu_ring_release(ring.h), "release")
        while True:
            rc = lib.pnetgpu_ring_wait(ring.h, ctypes.byref(rb))
            if rc == EEMPTY:
                break
            check(rc, "wait")
            frames += rb.n_frames
        el = time.perf_counter() - t0
    finally:
        ring.close()
        reg.close()
    return {"mpkts_s": round(frames / el / 1e6, 1), "link_gb_s": round(frames * (w.frame_len + 6 + 26) / el / 1e9, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="udp64")
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard(a.workload, bench.WORKLOADS[a.workload]["n"], 1000, dev)
    for r in range(a.rounds):
        p = bench.e2e_rate(sh, dev)
        z = bench.e2e_zero_copy_rate(sh, a.seconds, slots=a.slots)
        c = raw_zero_copy(lp, sh, a.seconds, a.slots)
        print(f"round {r}: e2e_pcie {p['link_gb_s']} GB/s  zero_copy (Ring.feed_region) {z['link_gb_s']} GB/s  "
              f"zero_copy (ctypes loop) {c['link_gb_s']} GB/s", flush=True)


if __name__ == "__main__":
    main()
