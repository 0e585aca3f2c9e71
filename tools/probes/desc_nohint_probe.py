#!/usr/bin/env python3
"""Kernel times of descriptor batches the mixed shape takes: the 1500-B UDP and
9000-B jumbo batches as compact descriptors without a size hint (bench.py's
descriptor line) and with it, and the IMIX batch (full record and verify-only). Used with tools/abvar.sh
(AB_SCRIPT) to compare library variants on one box.

  PNETGPU_LIB=.../libpnetgpu_V.so python tools/probes/desc_nohint_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
bench.load_library()
from bench import HBM_PEAK_GBS, Shard, descriptor_rate, time_launches  # noqa: E402


def nohint_only(name, n, dev, launches=5):
    """Only the no-hint descriptor batch of one workload, a few launches (a
    short program for rocprofv3 --pmc passes: tools/pmc_desc_nohint.sh)."""
    sh = Shard(name, n, 1000, dev)
    w = sh.w
    offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * np.uint64(w.stride)).astype(np.uint32).view(np.int32))
    offs = offs.to(dev)
    lens = torch.full((n,), w.frame_len, dtype=torch.int16, device=dev)
    res = bench.lp.RxResult(n, dev, bench.lp.IPV4_COLUMNS, counters=False)
    for _ in range(launches):
        bench.lp.rx_process(sh.data, offsets=offs, lengths=lens, out=res, flags=bench.lp.DESC_COMPACT)
    torch.cuda.synchronize()
    print(f"{name}: {launches} no-hint launches, alg bytes per launch {sh.frame_bytes + n * 32}", flush=True)
    return 0


def main():
    dev = torch.device("cuda", 0)
    if len(sys.argv) > 1 and sys.argv[1] == "--nohint-only":
        name = sys.argv[2]
        return nohint_only(name, {"udp1500": 1 << 20, "udp6_jumbo": 1 << 17}[name], dev)
    steps, warmup = 20, 3
    for name, n in (("udp1500", 1 << 20), ("udp6_jumbo", 1 << 17)):
        sh = Shard(name, n, 1000, dev)
        d = descriptor_rate(sh, steps, warmup, dev)
        for k in ("no_hint", "with_hint"):
            print(f"{name + '_desc':15s} {k:9s}: {d[k]['kernel_avg_ms'] * 1e3:7.1f} us  frac {d[k]['frac']:.4f}  "
                  f"{d[k]['kernel']}", flush=True)
        del sh
        torch.cuda.empty_cache()
    for name in ("imix", "imix_verify"):
        sh = Shard(name, 1 << 22, 1000, dev)
        s = torch.cuda.Stream(dev)
        ms = time_launches(lambda st: sh.step(st), steps, warmup, s)
        print(f"{name:15s}          : {ms * 1e3:7.1f} us  frac {sh.alg_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS:.4f}",
              flush=True)
        del sh
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
