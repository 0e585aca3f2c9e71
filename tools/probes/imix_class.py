#!/usr/bin/env python3
"""IMIX time attribution by frame class, one process, interleaved.

The bench's IMIX batch (2^22 frames, compact descriptors, 26-B record) is cut into
its three size classes. Each variant is timed over the same rounds:

  mixed            the whole batch, default kernel (what the bench line measures)
  sub<C>           only the C-byte frames, compact descriptors into the SAME buffer
                   (interleaved positions, the mixed kernel)
  packed<C>_desc   the C-byte frames copied back to back into their own buffer,
                   compact descriptors (mixed kernel)
  packed<C>_stride the same packed buffer in fixed-stride mode (small kernel for
                   64 B, MTU kernel for 576/1500 B): the class's shape ceiling

Batches of one class are smaller than the Infinity Cache could hold between
launches, so every timed launch is preceded by a 1-GiB read of an unrelated
tensor (cache flush) and timed by its own event pair (the same ~few-us event
overhead in every row). Output: one line per variant, median/min over rounds.

  python tools/probes/imix_class.py [--rounds 5] [--reps 6]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402

HBM = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--env", default="", help="KEY=v1,v2: extra variants of every row under that env value")
    ap.add_argument("--only", default="", help="comma list of variant-name prefixes to run")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = lp.synth.make("imix", a.n, seed=1000, corrupt_ppm=10000)
    buf = torch.from_numpy(w.buf).to(dev)
    offs_all = w.offsets.astype(np.uint64)
    lens_all = w.lengths.astype(np.uint32)
    flush = torch.ones(1 << 28, dtype=torch.float32, device=dev)   # 1 GiB
    s = torch.cuda.Stream(dev)

    variants = {}

    def add_desc(name, data, offs, lens, n_frame_bytes):
        do = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).to(dev)
        dl = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(dev)
        n = len(offs)
        res = lp.RxResult(n, dev, lp.IPV4_COLUMNS, counters=True)
        alg = n_frame_bytes + n * (26 + 6)

        def step(st, data=data, do=do, dl=dl, res=res):
            lp.rx_process(data, offsets=do, lengths=dl, out=res, stream=st, flags=lp.DESC_COMPACT)
        variants[name] = (step, alg, n, res)

    def add_stride(name, data, n, c):
        res = lp.RxResult(n, dev, lp.IPV4_COLUMNS, counters=True)
        alg = n * (c + 26)

        def step(st, data=data, n=n, c=c, res=res):
            lp.rx_process(data, stride=c, frame_len=c, n_frames=n, out=res, stream=st)
        variants[name] = (step, alg, n, res)

    add_desc("mixed", buf, offs_all, lens_all, int(lens_all.sum()))
    for c in (64, 576, 1500):
        sel = np.nonzero(lens_all == c)[0]
        add_desc(f"sub{c}", buf, offs_all[sel], lens_all[sel], int(len(sel)) * c)
        idx = (offs_all[sel][:, None] + np.arange(c, dtype=np.uint64)[None, :]).reshape(-1)
        packed = np.concatenate([w.buf[idx], np.zeros(32, np.uint8)])
        pd = torch.from_numpy(packed).to(dev)
        del idx, packed
        po = np.arange(len(sel), dtype=np.uint64) * np.uint64(c)
        add_desc(f"packed{c}_desc", pd, po, np.full(len(sel), c, np.uint32), len(sel) * c)
        add_stride(f"packed{c}_stride", pd, len(sel), c)
    if a.only:
        keep = tuple(a.only.split(","))
        variants = {k: v for k, v in variants.items() if k.startswith(keep)}

    key, vals = (a.env.split("=") + [""])[:2] if a.env else ("", "")
    envs = vals.split(",") if vals else [None]
    times = {(k, e): [] for k in variants for e in envs}
    for _ in range(a.rounds):
        for e in envs:
            if key:
                os.environ[key] = e
            for name, (step, alg, n, res) in variants.items():
                step(s)
                for _ in range(a.reps):
                    flush.sum()      # current stream; s waits for it below
                    s.wait_stream(torch.cuda.current_stream())
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    step(s)
                    e1.record(s)
                    s.synchronize()
                    times[(name, e)].append(e0.elapsed_time(e1))
    out = {}
    for (name, e), t in times.items():
        step, alg, n, res = variants[name]
        t = np.array(t)
        med = float(np.median(t))
        tag = name + (f" {key}={e}" if key else "")
        out[tag] = {"frames": n, "median_us": round(med * 1e3, 1), "min_us": round(float(t.min()) * 1e3, 1),
                    "alg_bytes": alg, "frac": round(alg / (med * 1e-3) / 1e9 / HBM, 4),
                    "ns_per_frame": round(med * 1e6 / n, 4)}
        print(f"{tag:28s} n={n:8d} median {med*1e3:8.1f} us  min {t.min()*1e3:8.1f} us  "
              f"{alg/(med*1e-3)/1e9:7.0f} GB/s ({alg/(med*1e-3)/1e9/HBM:.1%})  {med*1e6/n:.4f} ns/frame", flush=True)
    for e in envs:
        sfx = f" {key}={e}" if key else ""
        parts = [out.get(f"sub{c}{sfx}", {}).get("median_us") for c in (64, 576, 1500)]
        if all(p is not None for p in parts) and f"mixed{sfx}" in out:
            print(f"sum of class subsets{sfx}: {sum(parts):.1f} us vs mixed {out['mixed' + sfx]['median_us']:.1f} us",
                  flush=True)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
