#!/usr/bin/env python3
"""Times pnetgpu_checksum_slices_strided on the reference's bench shapes (20-B and
1024-B slices back to back, skipword 5) against the descriptor form, one process."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import libpnet_amd as lp  # noqa: E402

dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)


def timeit(fn, steps=20):
    for _ in range(3):
        fn()
    s.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(steps):
        fn()
    b.record(s)
    s.synchronize()
    return a.elapsed_time(b) / steps


# PROBE_SIZES: slice sizes (n = 2^29 / size); PROBE_BPC: grid sweep;
# PROBE_DENSE: PNETGPU_SLICE_DENSE_SPAN sweep (descriptor forms)
sizes = [int(x) for x in os.environ.get("PROBE_SIZES", "20,64,1024").split(",")]
for size, n in ((z, 1 << 24 if z <= 32 else (1 << 29) // z) for z in sizes):
    for bpc, dspan in ((b, ds) for b in os.environ.get("PROBE_BPC", "0").split(",")
                       for ds in os.environ.get("PROBE_DENSE", "").split(",")):
        lp.engine.apply_tuning_env({"PNETGPU_SLICE_BLOCKS_PER_CU": None if bpc == "0" else bpc,
                                    "PNETGPU_SLICE_DENSE_SPAN": dspan or None}, dev)
        print(f"blocks/CU {bpc} (0 = occupancy) dense span {dspan or 'default'}")
        d = torch.full((n * size + 32,), 99, dtype=torch.uint8, device=dev)
        offs = torch.arange(n, dtype=torch.int64, device=dev) * size
        lens = torch.full((n,), size, dtype=torch.int32, device=dev)
        sk = torch.full((n,), 5, dtype=torch.int32, device=dev)
        desc = lp.slice_descriptors(np.arange(n, dtype=np.uint64) * np.uint64(size), np.full(n, size),
                                    np.full(n, 5), device=dev)
        for _ in range(2):
            t_co = timeit(lambda: lp.checksum_slices_compact(d, desc, stream=s))
            t_st = timeit(lambda: lp.checksum_slices_strided(d, n, size, size, 5, stream=s))
            t_de = timeit(lambda: lp.checksum_slices(d, offs, lens, sk, stream=s))
            print(f"{size:5d}-B x {n}: strided {t_st*1e3:7.1f} us ({n*(size+2)/(t_st*1e-3)/8e12:.1%} of 8 TB/s)  "
                  f"descriptors {t_de*1e3:7.1f} us ({n*(size+18)/(t_de*1e-3)/8e12:.1%})  "
                  f"compact {t_co*1e3:7.1f} us ({n*(size+10)/(t_co*1e-3)/8e12:.1%})", flush=True)
        if os.environ.get("PROBE_ADV"):
            # ipv4_checksum_adv: each slice split into a main half and an extra half
            # (bytes: slice + 2 x 16-B descriptors + 8 addresses + 1 proto + 2 result)
            h = size // 2
            hl = torch.full((n,), h, dtype=torch.int32, device=dev)
            el = torch.full((n,), size - h, dtype=torch.int32, device=dev)
            ad = torch.zeros((n, 8), dtype=torch.uint8, device=dev)
            pr = torch.full((n,), 17, dtype=torch.uint8, device=dev)
            t_adv = timeit(lambda: lp.checksum_adv_slices(4, d, offs, hl, sk, offs + h, el, ad, pr, stream=s))
            print(f"{size:5d}-B x {n}: ipv4_checksum_adv halves {t_adv*1e3:7.1f} us "
                  f"({n*(size+2*16+8+1+2)/(t_adv*1e-3)/8e12:.1%})", flush=True)
