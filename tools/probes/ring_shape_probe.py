#!/usr/bin/env python3
"""Which of the ring's device stages slows its host push? The ring rebuilt from
parts — pnetgpu_batch_pack into four rotating pinned slots (64 MiB, 2^20 64-B
frames), each shipped on alternating streams once packed and reused after its
last stage is done — with the stages added one at a time: nothing shipped, the
H2D copy, + the receive kernel, + the D2H of its 26-B record. The push rate is
the time inside batch_pack; the real ring (push_many) runs last for reference.

    python tools/probes/ring_shape_probe.py [--rounds 2] [--seconds 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", 1 << 22, 1000, dev)
    offs, lens = bench._ring_source(sh)
    src = sh.w.buf
    n = 1 << 20
    slots = [torch.empty(64 << 20, dtype=torch.uint8).pin_memory() for _ in range(4)]
    sdesc = [(np.zeros(n, np.uint64), np.zeros(n, np.uint32)) for _ in range(4)]
    dslot = [torch.empty((64 << 20) + 32, dtype=torch.uint8, device=dev) for _ in range(2)]
    res = [lp.RxResult(n, dev, lp.IPV4_COLUMNS, counters=False) for _ in range(2)]
    hout = [torch.empty(res[0].nbytes, dtype=torch.uint8).pin_memory() for _ in range(4)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]

    def run(stage):
        done = [None] * 4
        frames = i = j = 0
        inside = 0.0
        t_start = time.perf_counter()
        while time.perf_counter() - t_start < a.seconds:
            q = j % 4
            if done[q] is not None:
                done[q].synchronize()
            t0 = time.perf_counter()
            k, _ = lp.batch_pack(src, offs[i:i + n], lens[i:i + n], slots[q].numpy(), *sdesc[q], check_bounds=False)
            inside += time.perf_counter() - t0
            if stage:
                s, d = streams[j % 2], j % 2
                with torch.cuda.stream(s):
                    dslot[d][:64 << 20].copy_(slots[q], non_blocking=True)
                    if stage >= 2:
                        lp.rx_process(dslot[d], stride=64, frame_len=64, n_frames=k, out=res[d], stream=s)
                    if stage >= 3:
                        res[d].to_host(hout[q], stream=s)
                    e = torch.cuda.Event()
                    e.record(s)
                    done[q] = e
            frames += k
            i = (i + k) % (len(offs) - n + 1)
            j += 1
        torch.cuda.synchronize()
        el = time.perf_counter() - t_start
        return {"push_gb_s": round(frames * 64 / inside / 1e9, 1), "frames_gb_s": round(frames * 64 / el / 1e9, 1)}

    cases = {"pack_only": lambda: run(0), "h2d": lambda: run(1), "h2d_kernel": lambda: run(2),
             "h2d_kernel_d2h": lambda: run(3),
             "real_ring": lambda: {"push_gb_s": bench.e2e_ring_rate(sh, seconds=a.seconds)["stages"]["push_gb_s"]}}
    out = {}
    for r in range(a.rounds):
        for k in (list(cases) if r % 2 == 0 else list(reversed(cases))):
            out.setdefault(k, []).append(cases[k]())
            print(json.dumps({"round": r, "case": k, **out[k][-1]}), flush=True)
    print(json.dumps({"summary": {k: [x["push_gb_s"] for x in v] for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
