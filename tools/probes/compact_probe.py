#!/usr/bin/env python3
"""IMIX (2^22 frames, descriptor mode, mixed kernel) with full u64/u32
descriptors vs PNETGPU_DESC_COMPACT u32/u16 ones: kernel time per launch
(HIP events around back-to-back launches on one stream), interleaved rounds,
records compared.

  python tools/probes/compact_probe.py [--n 4194304] [--reps 20]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402
from libpnet_amd.engine import IPV4_COLUMNS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = lp.synth.make("imix", a.n, seed=3)
    d = torch.from_numpy(w.buf).to(dev)
    cases = {
        "full": (torch.from_numpy(w.offsets.astype(np.int64)).to(dev),
                 torch.from_numpy(w.lengths.astype(np.int32)).to(dev), 0),
        "compact": (torch.from_numpy(w.offsets.astype(np.uint32).view(np.int32)).to(dev),
                    torch.from_numpy(w.lengths.astype(np.uint16).view(np.int16)).to(dev), lp.DESC_COMPACT),
    }
    s = torch.cuda.Stream()
    recs = {}
    for rnd in range(3):
        line = []
        for name, (o, l, fl) in cases.items():
            with torch.cuda.stream(s):
                res = lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, stream=s, flags=fl)
                for _ in range(2):
                    lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, out=res, stream=s, flags=fl)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, out=res, stream=s, flags=fl)
                e1.record(s)
            s.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            line.append(f"{name} {ms * 1e3:.1f} us ({a.n / ms / 1e3:.0f} Mpkts/s)")
            if rnd == 0:
                recs[name] = res.numpy()
        print(f"round {rnd}: " + "   ".join(line), flush=True)
    same = all(np.array_equal(recs["full"][c], recs["compact"][c]) for c in IPV4_COLUMNS)
    print("records identical:", same)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
