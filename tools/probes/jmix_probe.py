#!/usr/bin/env python3
"""Descriptor batches that mix minimum-size and jumbo frames (7 x 64-B UDP/IPv4
: 1 x 9000-B UDP/IPv6), the shape where whole-frame tail groups leave most of
a run's groups idle while one streams a jumbo frame. Times rx_process of the
same batch through the library PNETGPU_LIB names (run once per variant, e.g.
tools/abvar-style: default vs libpnetgpu_nosplit.so) and checks the records
against the oracle.

  PNETGPU_LIB=... python tools/probes/jmix_probe.py [--n 1048576]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402
from oracle import coracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n = a.n
    nj = n // 8
    small = lp.synth.make("udp64", n - nj, seed=7, corrupt_ppm=10000)
    jumbo = lp.synth.make("udp6_jumbo", nj, seed=8, corrupt_ppm=10000)
    buf = np.concatenate([small.buf[:(n - nj) * 64], jumbo.buf[:nj * jumbo.stride], np.zeros(64, np.uint8)])
    is_j = np.zeros(n, bool)
    is_j[7::8] = True
    offs = np.empty(n, np.uint64)
    lens = np.empty(n, np.uint32)
    offs[~is_j] = np.arange(n - nj, dtype=np.uint64) * 64
    lens[~is_j] = 64
    offs[is_j] = (n - nj) * 64 + np.arange(nj, dtype=np.uint64) * jumbo.stride
    lens[is_j] = jumbo.frame_len
    dev = torch.device("cuda", 0)
    d = torch.from_numpy(buf).to(dev)
    do = torch.from_numpy(offs.view(np.int64)).to(dev)
    dl = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = lp.RxResult(n, dev, lp.IPV4_COLUMNS)
    s = torch.cuda.Stream()
    for _ in range(3):
        lp.rx_process(d, offsets=do, lengths=dl, out=out, stream=s)
    s.synchronize()
    rec = coracle.rx_batch(buf, n, offsets=offs, lengths=lens, nthreads=16)
    got = out.numpy()
    bad = [c for c in lp.IPV4_COLUMNS if not np.array_equal(got[c], rec[c])]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        lp.rx_process(d, offsets=do, lengths=dl, out=out, stream=s)
    e1.record(s)
    s.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    alg = int(lens.sum()) + n * (26 + 12)
    print(f"jmix n={n} ({nj} jumbo): {ms * 1e3:.1f} us/launch, {alg / ms / 1e6:.0f} GB/s alg "
          f"({alg / ms / 1e6 / 8000:.1%} of 8 TB/s), kernel {lp.engine.last_rx_kernel()}, "
          f"records {'bit-exact' if not bad else 'MISMATCH ' + ','.join(bad)}", flush=True)


if __name__ == "__main__":
    main()
