#!/usr/bin/env python3
"""util::checksum descriptor batches of small packed slices through
slice_run_kernel and slice_tiny_kernel (tuning slice_kernel run / tiny), full
(16-B) and compact (8-B) descriptors, over slice sizes, interleaved rounds,
median kernel time per launch; also the tiny kernel with every run static
(static_pct 100). Every timed result is checked against the first kernel's.

  python tools/probes/tiny_probe.py [--sizes 8,12,16,20,24,32,48,64] [--rounds 3] [--variants run,tiny]
  tools/tiny_ab.sh TAG SIZES V...   the tiny kernel of library variants (PNETGPU_LIB), interleaved
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8,12,16,20,24,32,48,64")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--total", type=int, default=320 << 20, help="slice bytes per batch")
    ap.add_argument("--variants", default="run,tiny,tiny_static")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    variants = [("run", {"slice_kernel": "run"}), ("tiny", {"slice_kernel": "tiny"}),
                ("tiny_static", {"slice_kernel": "tiny", "static_pct": 100})]
    variants = [v for v in variants if v[0] in a.variants.split(",")]
    cases = []
    for size in (int(x) for x in a.sizes.split(",")):
        n = (a.total // size) // 64 * 64
        buf = torch.randint(0, 256, (n * size + 32,), dtype=torch.uint8, device=dev)
        offs = np.arange(n, dtype=np.uint64) * np.uint64(size)
        lens = np.full(n, size, np.uint32)
        skips = np.full(n, 5, np.uint32)
        do = torch.from_numpy(offs.view(np.int64)).to(dev)
        dl = torch.from_numpy(lens.view(np.int32)).to(dev)
        ds = torch.from_numpy(skips.view(np.int32)).to(dev)
        dc = lp.slice_descriptors(offs, lens, skips, device=dev)
        cases.append((size, "full", n, size + 16 + 2,
                      lambda b=buf, o=do, ln=dl, k=ds: lp.checksum_slices(b, o, ln, k, stream=s)))
        cases.append((size, "compact", n, size + 8 + 2,
                      lambda b=buf, c=dc: lp.checksum_slices_compact(b, c, stream=s)))
    times = {}
    ref = {}
    for r in range(a.rounds):
        for size, form, n, alg, fn in cases:
            for name, tune in variants:
                with lp.engine.tuning(0, **tune):
                    out = fn()
                    s.synchronize()
                    key = (size, form)
                    got = out.cpu()
                    if key not in ref:
                        ref[key] = got
                    assert torch.equal(got, ref[key]), (size, form, name)
                    fn()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for _ in range(10):
                        fn()
                    e1.record(s)
                    s.synchronize()
                    times.setdefault((size, form, name), []).append(e0.elapsed_time(e1) / 10)
        print(f"round {r} done", file=sys.stderr, flush=True)
    print(f"{'size':>5} {'form':8} {'kernel':12} {'us':>8} {'Mslices/s':>10} {'frac':>6}")
    for size, form, n, alg, fn in cases:
        for name, _ in variants:
            ms = float(np.median(times[(size, form, name)]))
            print(f"{size:5d} {form:8} {name:12} {ms * 1e3:8.1f} {n / ms / 1e3:10.0f} "
                  f"{n * alg / ms / 1e6 / PEAK:6.3f}", flush=True)


if __name__ == "__main__":
    main()
