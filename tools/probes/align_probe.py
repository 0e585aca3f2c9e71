#!/usr/bin/env python3
"""Does the IMIX kernel pay for 128-B lines shared by neighbouring frames?
The same IMIX frames timed packed (as generated) and re-packed at 128-B aligned
offsets (no line holds two frames; algorithmic bytes unchanged), both in
descriptor mode through the mixed kernel.

  python tools/probes/align_probe.py [--n 4194304] [--reps 20]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402
from libpnet_amd.engine import IPV4_COLUMNS  # noqa: E402


def repack(buf, offs, lens, align):
    """Copy every frame to an `align`-aligned offset (vectorised per frame length)."""
    span = (lens.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    noffs = np.concatenate([[0], np.cumsum(span)[:-1]]).astype(np.uint64)
    out = np.zeros(int(span.sum()) + 64, np.uint8)
    for L in np.unique(lens):
        idx = np.nonzero(lens == L)[0]
        for c in range(0, len(idx), 1 << 15):
            ii = idx[c:c + (1 << 15)]
            src = offs[ii].astype(np.int64)[:, None] + np.arange(int(L))[None, :]
            dst = noffs[ii].astype(np.int64)[:, None] + np.arange(int(L))[None, :]
            out[dst] = buf[src]
    return out, noffs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = lp.synth.make("imix", a.n, seed=3)
    abuf, aoffs = repack(w.buf, w.offsets, w.lengths, 128)
    cases = {}
    for name, buf, offs in (("packed", w.buf, w.offsets), ("aligned128", abuf, aoffs)):
        cases[name] = (torch.from_numpy(buf).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev),
                       torch.from_numpy(w.lengths.view(np.int32)).to(dev))
    s = torch.cuda.Stream()
    ref = None
    for rnd in range(3):
        line = []
        for name, (d, o, l) in cases.items():
            with torch.cuda.stream(s):
                res = lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, stream=s)
                for _ in range(2):
                    lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, out=res, stream=s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    lp.rx_process(d, offsets=o, lengths=l, columns=IPV4_COLUMNS, out=res, stream=s)
                e1.record(s)
            s.synchronize()
            if rnd == 0:   # the same frames must give the same records wherever they sit
                got = {c: v for c, v in res.numpy().items() if c != "l4_offset"}
                if ref is None:
                    ref = got
                else:
                    same = all(np.array_equal(ref[c], got[c]) for c in ref)
                    print(f"records equal packed vs aligned: {same}", flush=True)
            line.append(f"{name} {e0.elapsed_time(e1) / a.reps * 1e3:6.1f} us")
        print(f"round {rnd}: " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
