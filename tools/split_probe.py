#!/usr/bin/env python3
"""Timing probe for a size-class split of the IMIX batch (no new kernel): the
same frames handed over as two descriptor batches - short frames (window only)
and long frames - each with dense result columns, under the existing kernels
(PNETGPU_RX_KIND picks the long batch's shape). If short + long is not clearly
below the fused mixed kernel, a device-side split cannot win either (it would
add a classification pass and scattered column writes on top).

  python tools/split_probe.py [--n 4194304] [--reps 20]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    offs, lens = w.offsets, w.lengths
    short = lens <= 113          # whole frame inside the 128-B window at any alignment
    sets = {
        "all": (offs, lens),
        "short": (offs[short], lens[short]),
        "long": (offs[~short], lens[~short]),
    }
    dsets = {k: (torch.from_numpy(o.view(np.int64)).to(dev), torch.from_numpy(l.view(np.int32)).to(dev))
             for k, (o, l) in sets.items()}
    s = torch.cuda.Stream()

    def run(key, kind):
        if kind is None:
            os.environ.pop("PNETGPU_RX_KIND", None)
        else:
            os.environ["PNETGPU_RX_KIND"] = str(kind)
        o, l = dsets[key]
        res = None
        with torch.cuda.stream(s):
            for _ in range(3):
                res = lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, stream=s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, out=res, stream=s)
            e1.record(s)
        s.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    cases = [("all", None), ("short", None), ("long", None), ("long", 2), ("long", 3)]
    for rnd in range(3):
        t = {f"{k}/kind={kind}": run(k, kind) for k, kind in cases}
        print(f"round {rnd}: " + "  ".join(f"{k} {v:6.1f} us" for k, v in t.items()), flush=True)
        best_long = min(t["long/kind=None"], t["long/kind=2"], t["long/kind=3"])
        print(f"  short + best long = {t['short/kind=None'] + best_long:6.1f} us vs fused {t['all/kind=None']:6.1f} us "
              f"(frames: {int(short.sum())} short, {int((~short).sum())} long)", flush=True)


if __name__ == "__main__":
    main()
