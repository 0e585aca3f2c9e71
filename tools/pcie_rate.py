"""Raw PCIe copy rates on this box (pinned host <-> HBM), to price bench.py's
PCIe-inclusive lines: H2D alone, D2H alone, both directions at once, for chunk
sizes 4-256 MiB on one or two streams."""
import time

import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    dev = torch.device("cuda", 0)
    total = 1 << 30
    h = torch.empty(total, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(total, dtype=torch.uint8).pin_memory()
    d = torch.empty(total, dtype=torch.uint8, device=dev)
    d2 = torch.empty(total, dtype=torch.uint8, device=dev)
    ss = [torch.cuda.Stream(dev) for _ in range(4)]
    for chunk_mib in (4, 16, 64, 256):
        ch = chunk_mib << 20
        nch = total // ch
        for nst in (1, 2, 4):
            def h2d():
                for k in range(nch):
                    with torch.cuda.stream(ss[k % nst]):
                        d[k * ch:(k + 1) * ch].copy_(h[k * ch:(k + 1) * ch], non_blocking=True)

            def d2h():
                for k in range(nch):
                    with torch.cuda.stream(ss[k % nst]):
                        h2[k * ch:(k + 1) * ch].copy_(d2[k * ch:(k + 1) * ch], non_blocking=True)

            def both():
                h2d()
                d2h()
            print(f"chunk {chunk_mib:4d} MiB streams {nst}: H2D {rate(h2d, total):6.1f} GB/s  "
                  f"D2H {rate(d2h, total):6.1f} GB/s  both {rate(both, 2 * total):6.1f} GB/s (sum)", flush=True)


if __name__ == "__main__":
    main()
