#!/usr/bin/env python3
"""Why the ring's push runs slower than pnetgpu_batch_pack alone: the same pack
(2^20 64-B frames, 16 threads) into destinations allocated different ways —
hipHostMalloc with the ring's flags (hipHostMallocDefault), torch's pinned
allocator, plain pageable numpy — with its descriptor arrays in pageable or
pinned memory. One process, interleaved rounds; GB/s of frame bytes.

    python tools/probes/pinned_write_probe.py [--rounds 3]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import libpnet_amd as lp  # noqa: E402


def hip_host_malloc(nbytes, flags):
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    hip.hipHostMalloc.restype = ctypes.c_int
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    p = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(p), nbytes, flags)
    assert rc == 0, rc
    return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=1.0)
    a = ap.parse_args()
    torch.cuda.init()
    n = 1 << 20
    w = lp.synth.make("udp64", 4 * n, seed=3)
    offs = np.arange(4 * n, dtype=np.uint64) * np.uint64(64)
    lens = np.full(4 * n, 64, np.uint32)
    dsts = {
        "hipHostMalloc": hip_host_malloc(64 << 20, 0),
        "torch_pinned": torch.empty(64 << 20, dtype=torch.uint8).pin_memory().numpy(),
        "pageable": np.zeros(64 << 20, np.uint8),
    }
    descs = {
        "pageable": (np.zeros(n, np.uint64), np.zeros(n, np.uint32)),
        "hipHostMalloc": (hip_host_malloc(8 * n, 0).view(np.uint64), hip_host_malloc(4 * n, 0).view(np.uint32)),
    }
    for d in dsts.values():
        d[:] = 1                                     # touched once before timing
    out = {}
    for r in range(a.rounds):
        for dn, dst in dsts.items():
            for en, (do, dl) in descs.items():
                key = f"dst={dn} desc={en}"
                frames = i = 0
                t0 = time.perf_counter()
                while time.perf_counter() - t0 < a.seconds:
                    k, _ = lp.batch_pack(w.buf, offs[i:i + n], lens[i:i + n], dst, do, dl, check_bounds=False)
                    frames += k
                    i = (i + k) % (4 * n)
                el = time.perf_counter() - t0
                out.setdefault(key, []).append(round(frames * 64 / el / 1e9, 1))
                print(json.dumps({"round": r, "case": key, "gb_s": out[key][-1]}), flush=True)
    # The same pack while host->device DMA reads another pinned buffer (what the
    # ring's push overlaps with), and the DMA's own rate with and without it.
    dev = torch.device("cuda", 0)
    src = torch.empty(64 << 20, dtype=torch.uint8).pin_memory()
    dst_d = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)

    def dma(copies):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            for _ in range(copies):
                dst_d.copy_(src, non_blocking=True)
            e1.record(s)
        return e0, e1, copies * (64 << 20)

    dst, (do, dl) = dsts["hipHostMalloc"], descs["hipHostMalloc"]
    for r in range(a.rounds):
        e0, e1, nb = dma(300)
        e1.synchronize()
        out.setdefault("dma_alone", []).append(round(nb / (e0.elapsed_time(e1) / 1e3) / 1e9, 1))
        e0, e1, nb = dma(900)
        frames = i = 0
        t0 = time.perf_counter()
        while not e1.query():
            k, _ = lp.batch_pack(w.buf, offs[i:i + n], lens[i:i + n], dst, do, dl, check_bounds=False)
            frames += k
            i = (i + k) % (4 * n)
        el = time.perf_counter() - t0
        out.setdefault("pack_during_dma", []).append(round(frames * 64 / el / 1e9, 1))
        out.setdefault("dma_during_pack", []).append(round(nb / (e0.elapsed_time(e1) / 1e3) / 1e9, 1))
        print(json.dumps({"round": r, **{k: out[k][-1] for k in ("dma_alone", "pack_during_dma",
                                                                  "dma_during_pack")}}), flush=True)
    # The ring's shape rebuilt from parts: pack into 4 rotating pinned slots
    # (64 MiB each), each shipped H2D on alternating streams once full, a slot
    # reused after its copy is done; `ship` off packs the same rotation alone.
    slots = [hip_host_malloc(64 << 20, 0) for _ in range(4)]
    sdesc = [(hip_host_malloc(8 * n, 0).view(np.uint64), hip_host_malloc(4 * n, 0).view(np.uint32))
             for _ in range(4)]
    dslot = [torch.empty(64 << 20, dtype=torch.uint8, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    tslot = [torch.from_numpy(x) for x in slots]
    for r in range(a.rounds):
        for ship in (False, True):
            done = [None] * 4
            frames = i = j = 0
            inside = 0.0
            t_start = time.perf_counter()
            while time.perf_counter() - t_start < a.seconds:
                q = j % 4
                if done[q] is not None:
                    done[q].synchronize()
                t0 = time.perf_counter()
                k, _ = lp.batch_pack(w.buf, offs[i:i + n], lens[i:i + n], slots[q], *sdesc[q], check_bounds=False)
                inside += time.perf_counter() - t0
                if ship:
                    s = streams[j % 2]
                    with torch.cuda.stream(s):
                        dslot[j % 2].copy_(tslot[q], non_blocking=True)
                        e = torch.cuda.Event()
                        e.record(s)
                        done[q] = e
                frames += k
                i = (i + k) % (4 * n)
                j += 1
            torch.cuda.synchronize()
            el = time.perf_counter() - t_start
            key = "ring_shape_" + ("shipped" if ship else "pack_only")
            out.setdefault(key, []).append({"push_gb_s": round(frames * 64 / inside / 1e9, 1),
                                            "wall_gb_s": round(frames * 64 / el / 1e9, 1)})
            print(json.dumps({"round": r, "case": key, **out[key][-1]}), flush=True)

    # The same pack after the pool sat idle (the ring's push follows a wait on
    # the oldest batch): only the time inside batch_pack is counted.
    for r in range(a.rounds):
        for idle_us in (0, 100, 500, 2000):
            frames = i = 0
            inside = 0.0
            t_end = time.perf_counter() + a.seconds
            while time.perf_counter() < t_end:
                if idle_us:
                    time.sleep(idle_us / 1e6)
                t0 = time.perf_counter()
                k, _ = lp.batch_pack(w.buf, offs[i:i + n], lens[i:i + n], dst, do, dl, check_bounds=False)
                inside += time.perf_counter() - t0
                frames += k
                i = (i + k) % (4 * n)
            key = f"pack_after_idle_{idle_us}us"
            out.setdefault(key, []).append(round(frames * 64 / inside / 1e9, 1))
            print(json.dumps({"round": r, "case": key, "gb_s": out[key][-1]}), flush=True)
    print(json.dumps({"summary": out, "host_threads": lp.host_threads()}), flush=True)


if __name__ == "__main__":
    main()
