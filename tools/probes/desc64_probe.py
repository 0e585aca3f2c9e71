import sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import libpnet_amd as lp
import bench
bench.load_library()

dev = torch.device("cuda", 0)
n = 1 << 24
w = lp.synth.make("udp64", n, seed=5, corrupt_ppm=10000)
s = torch.cuda.Stream(dev)

def timeit(fn, steps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(steps): fn()
    b.record(s); s.synchronize()
    return a.elapsed_time(b) / steps

for gap in (0, 16):
    stride = 64 + gap
    buf = np.zeros(n * stride + 64, np.uint8)
    src = w.buf[: n * 64].reshape(n, 64)
    buf[: n * stride].reshape(n, stride)[:, :64] = src
    d = torch.from_numpy(buf).to(dev)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * stride
    lens = torch.full((n,), 64, dtype=torch.int32, device=dev)
    out = lp.RxResult(n, dev, lp.IPV4_COLUMNS, counters=True)
    t_desc = timeit(lambda: lp.rx_process(d, offsets=offs, lengths=lens, out=out, stream=s))
    t_strd = timeit(lambda: lp.rx_process(d, stride=stride, frame_len=64, n_frames=n, out=out, stream=s))
    print(f"gap {gap:2d}: descriptor mode {t_desc:.4f} ms, fixed stride {t_strd:.4f} ms", flush=True)

# 60-B frames packed back to back (the captured TCP frame of bench_ipv4_parsing,
# packet_benchmarks.rs:63): frame starts at every 4-B alignment
frame = np.frombuffer(bench.CAPTURED_TCP_FRAME, np.uint8)
buf = np.concatenate([np.tile(frame, n), np.zeros(64, np.uint8)])
d = torch.from_numpy(buf).to(dev)
offs = torch.arange(n, dtype=torch.int64, device=dev) * len(frame)
lens = torch.full((n,), len(frame), dtype=torch.int32, device=dev)
out = lp.RxResult(n, dev, lp.IPV4_COLUMNS, counters=True)
t_desc = timeit(lambda: lp.rx_process(d, offsets=offs, lengths=lens, out=out, stream=s))
print(f"60-B packed: descriptor mode {t_desc:.4f} ms", flush=True)
