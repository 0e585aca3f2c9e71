#!/usr/bin/env python3
"""Times the batched util::checksum / ipv4_checksum slice entry points on the
reference's bench shapes (20-B and 1024-B slices, skipword 5) and on 1466-B
TCP segments, median of interleaved rounds (same-box A/B with PNETGPU_LIB)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream()
    cases = []
    for name, size, n, pseudo in (("small20", 20, 1 << 24, False), ("large1024", 1024, 1 << 20, False),
                                  ("tcp1466_v4", 1466, 1 << 20, True)):
        buf = torch.randint(0, 256, (n * size + 32,), dtype=torch.uint8, device=dev)
        offs = torch.arange(n, dtype=torch.int64, device=dev) * size
        lens = torch.full((n,), size, dtype=torch.int32, device=dev)
        skips = torch.full((n,), 5 if not pseudo else 8, dtype=torch.int32, device=dev)
        addrs = torch.randint(0, 256, (n, 8), dtype=torch.uint8, device=dev)
        protos = torch.full((n,), 6, dtype=torch.uint8, device=dev)
        fn = ((lambda b=buf, o=offs, ln=lens, k=skips, ad=addrs, pr=protos:
               lp.ipv4_checksum_slices(b, o, ln, k, ad, pr, stream=s)) if pseudo else
              (lambda b=buf, o=offs, ln=lens, k=skips: lp.checksum_slices(b, o, ln, k, stream=s)))
        cases.append((name, n, size, fn))
    # the 20-B shape through 8-B compact descriptors, and descriptor slices of 64 / 256 B
    cbuf = torch.randint(0, 256, ((1 << 24) * 20 + 32,), dtype=torch.uint8, device=dev)
    n = 1 << 24
    cdesc = lp.slice_descriptors(np.arange(n, dtype=np.uint64) * 20, np.full(n, 20, np.uint32),
                                 np.full(n, 5, np.uint32), device=dev)
    cases.append(("small20_compact", n, 20, lambda b=cbuf, dc=cdesc: lp.checksum_slices_compact(b, dc, stream=s)))
    for size, n in ((64, 1 << 23), (256, 1 << 22)):
        buf = torch.randint(0, 256, (n * size + 32,), dtype=torch.uint8, device=dev)
        offs = torch.arange(n, dtype=torch.int64, device=dev) * size
        lens = torch.full((n,), size, dtype=torch.int32, device=dev)
        skips = torch.full((n,), 5, dtype=torch.int32, device=dev)
        cases.append((f"d{size}", n, size, lambda b=buf, o=offs, ln=lens, k=skips: lp.checksum_slices(b, o, ln, k,
                                                                                                   stream=s)))
    # the reference's 20-B shape as uniform slices (no descriptors)
    sbuf = torch.randint(0, 256, ((1 << 24) * 20 + 32,), dtype=torch.uint8, device=dev)
    cases.append(("strided20", 1 << 24, 20,
                  lambda b=sbuf: lp.checksum_slices_strided(b, 1 << 24, 20, 20, 5, stream=s)))
    # --env KEY=v1,v2 (e.g. PNETGPU_STATIC_PCT=100,90): every case per value, interleaved
    env = next((x.split("=", 1) for x in sys.argv[1:] if "=" in x), None)
    vals = env[1].split(",") if env else [None]
    cases = [(f"{name}{'' if v is None else ' ' + env[0] + '=' + v}", n, size, fn, v)
             for name, n, size, fn in cases for v in vals]
    times = {c[0]: [] for c in cases}
    for _ in range(3):
        for name, n, size, fn, v in cases:
            if v is not None:
                lp.engine.apply_tuning_env({env[0]: v}, dev)
            for _ in range(2):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(10):
                fn()
            b.record(s)
            s.synchronize()
            times[name].append(a.elapsed_time(b) / 10)
    for name, n, size, fn, v in cases:
        ms = float(np.median(times[name]))
        print(f"{name:36s} {ms * 1e3:8.1f} us  {n / ms / 1e6:9.1f} Mslices/s  "
              f"{n * (size + 18) / ms / 1e6:7.0f} GB/s alg", flush=True)


if __name__ == "__main__":
    main()
