"""Wall time per step of the 64-B bench step three ways, same box: per-step
HIP events around each launch (bench.py's kernel timing), plain back-to-back
launches, and the K launches captured once in a HIP graph and replayed."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
bench.load_library()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    sh = bench.Shard("udp64", bench.WORKLOADS["udp64"]["n"], 1000, dev)
    s = torch.cuda.Stream(dev)
    for rep in range(3):
        wall, kern = bench.time_shard(sh, steps, 3, s, False)
        print(f"events   : {wall / steps * 1e3:.4f} ms/step, kernel avg {sum(kern) / len(kern):.4f}")
        for _ in range(3):
            sh.step(s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            sh.step(s)
        torch.cuda.synchronize()
        print(f"plain    : {(time.perf_counter() - t0) / steps * 1e3:.4f} ms/step")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            sh.step(s)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(steps):
                    sh.step(torch.cuda.current_stream())
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        print(f"graph    : {(time.perf_counter() - t0) / steps * 1e3:.4f} ms/step")
        del g


if __name__ == "__main__":
    main()
