#!/usr/bin/env python3
"""Is the ring's own pinned slot memory slower for the host pack to write than
other memory? The pack (pnetgpu_batch_pack, 2^20 64-B frames) into the real
ring's four slot batches — their pointers taken from waited copy=False batches,
written while the ring is idle — against torch-pinned and pageable buffers, one
process, interleaved rounds; then the push_many rate inside the running ring.

    python tools/probes/ring_slot_write_probe.py [--rounds 3]
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
import bench  # noqa: E402


def pack_rate(lp, src, offs, lens, dst, seconds):
    n = 1 << 20
    do, dl = np.zeros(n, np.uint64), np.zeros(n, np.uint32)
    frames = i = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        k, _ = lp.batch_pack(src, offs[i:i + n], lens[i:i + n], dst, do, dl, check_bounds=False)
        frames += k
        i = (i + k) % (len(offs) - n + 1)
    return round(frames * 64 / (time.perf_counter() - t0) / 1e9, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=1.0)
    a = ap.parse_args()
    lp = bench.load_library()
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", 1 << 22, 1000, dev)
    offs, lens = bench._ring_source(sh)
    src = sh.w.buf
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=False)
    slots = {}
    for b in list(ring.feed_many(src, offs, lens)) + list(ring.drain()):
        slots[int(b._ptr[2])] = True            # the slot's pinned batch (copy=False)
    views = [np.ctypeslib.as_array((ctypes.c_uint8 * (64 << 20)).from_address(p)) for p in slots]
    dsts = {f"ring_slot{k}": v for k, v in enumerate(views)}
    dsts["torch_pinned"] = torch.empty(64 << 20, dtype=torch.uint8).pin_memory().numpy()
    dsts["pageable"] = np.ones(64 << 20, np.uint8)
    # numpy's large arrays are madvise'd for transparent huge pages; the same
    # kind of buffer page-locked and mapped for DMA (pnetgpu_host_register)
    dsts["pageable_registered"] = np.ones(64 << 20, np.uint8)
    reg = lp.HostRegistration(dsts["pageable_registered"])
    out = {}
    for r in range(a.rounds):
        for k in (list(dsts) if r % 2 == 0 else list(reversed(dsts))):
            out.setdefault(k, []).append(pack_rate(lp, src, offs, lens, dsts[k], a.seconds))
            print(json.dumps({"round": r, "dst": k, "gb_s": out[k][-1]}), flush=True)
    # the same ring running (its push_many rate from its statistics)
    ring.reset_stats()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        for b in ring.feed_many(src, offs, lens):
            del b
    for b in ring.drain():
        del b
    st = ring.stats()
    out["ring_push_gb_s"] = round(st["bytes"] / (st["push_ns"] / 1e9) / 1e9, 1)
    out["ring_wait_s"] = round(st["wait_ns"] / 1e9, 3)
    ring.close()
    reg.close()
    print(json.dumps({"summary": out, "slots_seen": len(slots)}), flush=True)


if __name__ == "__main__":
    main()
