#!/usr/bin/env python3
"""Why the copying ring moves fewer link bytes than the zero-copy ring when its
push alone is not the bound (profiles/r06/e2e/): the zero-copy ring (the
bench's e2e_zero_copy) with one factor changed at a time, one process,
interleaved rounds, 64-B frames.

  zc            e2e_zero_copy: region in a hipHostRegister'd numpy buffer
  zc_hostmalloc the same frames in hipHostMalloc'd memory (the ring's slots' kind)
  zc_memload    zc while 8 Python threads stream numpy copies through host
                memory (~the push's traffic; numpy releases the GIL)
  ring          e2e_ring (the copying producer)

    python tools/probes/ring_dma_probe.py [--rounds 2] [--seconds 2]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def hip_host_malloc(nbytes):
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    hip.hipHostMalloc.restype = ctypes.c_int
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), nbytes, 0) == 0
    return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))


def zc_from(lp, buf, offs, lens, seconds, register):
    reg = lp.HostRegistration(buf) if register else None
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=False, stage_times=True)
    frames = 0
    try:
        bench._ring_warm(ring, lambda: ring.feed_region(buf, offs, lens))
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for b in ring.feed_region(buf, offs, lens):
                frames += b.n
                del b
        for b in ring.drain():
            frames += b.n
        el = time.perf_counter() - t0
        st = bench._ring_stages(ring, el)
    finally:
        ring.close()
        if reg:
            reg.close()
    return {"link_gb_s": round(frames * (64 + 6 + 26) / el / 1e9, 2), "wait_s": st["wait_s"],
            "h2d_gb_s": st.get("h2d_gb_s")}


class MemLoad:
    def __init__(self, threads=8, mib=64):
        self.stop = False
        self.bytes = 0
        self.src = [np.ones(mib << 20, np.uint8) for _ in range(threads)]
        self.dst = [np.zeros(mib << 20, np.uint8) for _ in range(threads)]
        self.th = [threading.Thread(target=self.run, args=(t,)) for t in range(threads)]

    def run(self, t):
        while not self.stop:
            np.copyto(self.dst[t], self.src[t])
            self.bytes += self.src[t].size

    def __enter__(self):
        self.t0 = time.perf_counter()
        for t in self.th:
            t.start()
        return self

    def __exit__(self, *a):
        self.stop = True
        for t in self.th:
            t.join()
        self.rate = round(2 * self.bytes / (time.perf_counter() - self.t0) / 1e9, 1)   # read + write


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", 1 << 22, 1000, dev)
    offs, lens = bench._ring_source(sh)
    span = int(offs[-1] + lens[-1])
    reg_buf = sh.w.buf[:span]
    hm = hip_host_malloc(span)
    hm[:] = reg_buf

    def memload():
        with MemLoad() as m:
            r = zc_from(lp, reg_buf, offs, lens, a.seconds, True)
        r["memload_gb_s"] = m.rate
        return r

    cases = {
        "zc": lambda: zc_from(lp, reg_buf, offs, lens, a.seconds, True),
        "zc_hostmalloc": lambda: zc_from(lp, hm, offs, lens, a.seconds, False),
        "zc_memload": memload,
        "ring": lambda: {k: v for k, v in bench.e2e_ring_rate(sh, seconds=a.seconds).items()
                         if k in ("link_gb_s", "stages")},
    }
    out = {k: [] for k in cases}
    for r in range(a.rounds):
        for k in (list(cases) if r % 2 == 0 else list(reversed(cases))):
            out[k].append(cases[k]())
            print(json.dumps({"round": r, "case": k, **out[k][-1]}), flush=True)
    print(json.dumps({"summary": {k: [x["link_gb_s"] for x in v] for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
