#!/usr/bin/env python3
"""Why the pinned ring moves fewer link bytes than the plain pipeline
(bench.py e2e_ring vs e2e_pcie): the same 64-B frames through pipelines that
differ in one factor each, one process, interleaved rounds. All ship the
frames host -> device, run the receive kernel and copy the 26-B record back.

  pcie2      bench.e2e_rate: 2 streams, every chunk enqueued up front
  pcie4      the same on 4 streams
  depth2     2 streams, at most 2 chunks in flight (the ring's consumer waits
             for the oldest before it enqueues the next)
  depth2d    depth2 + compact descriptors shipped and a descriptor-mode kernel
             (what every ring batch does)
  ring       the real ring (pnetgpu_ring_push_many), stage timing off / on
  zero_copy  the real zero-copy ring, stage timing off

    python tools/ring_factor_probe.py [--rounds 2] [--seconds 2] [--cases depth2,ring,...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def pipeline(lp, sh, dev, nstreams, depth, desc, seconds, chunks=16, stagger=False):
    w = sh.w
    n, stride = sh.n, w.stride
    per = n // chunks
    host = torch.from_numpy(w.buf[: n * stride]).pin_memory()
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    nb = max(nstreams, depth or 2)
    dbuf = [torch.empty(per * stride + 32, dtype=torch.uint8, device=dev) for _ in range(nb)]
    res = [lp.RxResult(per, dev, lp.IPV4_COLUMNS, counters=False) for _ in range(nb)]
    hout = [torch.empty(r.nbytes, dtype=torch.uint8).pin_memory() for r in res]
    if desc:
        h_off = torch.from_numpy((np.arange(per, dtype=np.uint64) * np.uint64(stride)).astype(np.uint32)
                                 .view(np.int32)).pin_memory()
        h_len = torch.from_numpy(np.full(per, stride, np.uint16).view(np.int16)).pin_memory()
        d_off = [torch.empty(per, dtype=torch.int32, device=dev) for _ in range(nb)]
        d_len = [torch.empty(per, dtype=torch.int16, device=dev) for _ in range(nb)]
    done = [None] * nb
    up = [None] * nb

    def chunk(i):
        j = i % nb
        s = streams[i % nstreams]
        if depth and done[j] is not None:
            done[j].synchronize()                  # the consumer waits for this buffer's previous chunk
        k = i % chunks
        with torch.cuda.stream(s):
            dbuf[j][: per * stride].copy_(host[k * per * stride:(k + 1) * per * stride], non_blocking=True)
            u = torch.cuda.Event()
            u.record(s)
            up[j] = u
            if desc:
                d_off[j].copy_(h_off, non_blocking=True)
                d_len[j].copy_(h_len, non_blocking=True)
                lp.rx_process(dbuf[j], offsets=d_off[j], lengths=d_len[j], out=res[j], stream=s,
                              flags=lp.DESC_COMPACT)
            else:
                lp.rx_process(dbuf[j], stride=stride, frame_len=stride, n_frames=per, out=res[j], stream=s)
            res[j].to_host(hout[j], stream=s)
            ev = torch.cuda.Event()
            ev.record(s)
            done[j] = ev

    for i in range(2 * chunks):
        chunk(i)
    torch.cuda.synchronize()
    i, t0 = 0, time.perf_counter()
    if stagger:                                     # the second stream starts one upload behind the first
        chunk(i)
        up[i % nb].synchronize()
        i += 1
    while time.perf_counter() - t0 < seconds:
        for _ in range(chunks):
            chunk(i)
            i += 1
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    up = stride + (6 if desc else 0)
    return round(i * per * (up + 26) / el / 1e9, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--cases", default="", help="comma list (default: all)")
    ap.add_argument("--frames", type=int, default=1 << 22, help="batch frames (16 chunks of them)")
    a = ap.parse_args()
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", a.frames, 1000, dev)
    mib = sh.n * 64 // 16 >> 20                     # chunk MiB at 16 chunks
    cases = {
        "pcie2": lambda: pipeline(lp, sh, dev, 2, 0, False, a.seconds),
        "pcie4": lambda: pipeline(lp, sh, dev, 4, 0, False, a.seconds),
        "depth2": lambda: pipeline(lp, sh, dev, 2, 2, False, a.seconds),
        "depth2d": lambda: pipeline(lp, sh, dev, 2, 2, True, a.seconds),
        "depth3d": lambda: pipeline(lp, sh, dev, 3, 3, True, a.seconds),
        "depth2_stagger": lambda: pipeline(lp, sh, dev, 2, 2, False, a.seconds, stagger=True),
        "depth2_x4": lambda: pipeline(lp, sh, dev, 2, 2, False, a.seconds, chunks=64),   # chunks a quarter the size
        "pcie2_x4": lambda: pipeline(lp, sh, dev, 2, 0, False, a.seconds, chunks=64),
        "bench_e2e": lambda: bench.e2e_rate(sh, dev, seconds=a.seconds)["link_gb_s"],
        "bench_e2e_one_prio": lambda: bench.e2e_rate(sh, dev, seconds=a.seconds, priorities=False)["link_gb_s"],
        "prio_info": lambda: list(torch.cuda.Stream.priority_range()),
        "bench_e2e_d3": lambda: bench.e2e_rate(sh, dev, seconds=a.seconds, depth=3)["link_gb_s"],
        "bench_e2e_d2": lambda: bench.e2e_rate(sh, dev, seconds=a.seconds, depth=2)["link_gb_s"],
        "ring": lambda: bench.e2e_ring_rate(sh, seconds=a.seconds, stage_times=False)["link_gb_s"],
        "ring_timed": lambda: bench.e2e_ring_rate(sh, seconds=a.seconds)["link_gb_s"],
        "zero_copy": lambda: bench.e2e_zero_copy_rate(sh, seconds=a.seconds, stage_times=False)["link_gb_s"],
    }
    if a.cases:
        cases = {k: v for k, v in cases.items() if k in a.cases.split(",")}
    out = {k: [] for k in cases}
    for r in range(a.rounds):
        order = list(cases) if r % 2 == 0 else list(reversed(cases))
        for k in order:
            out[k].append(cases[k]())
            print(json.dumps({"round": r, "case": k, "link_gb_s": out[k][-1], "chunk_mib": mib}), flush=True)
    print(json.dumps({"summary": out}), flush=True)


if __name__ == "__main__":
    main()
