#!/usr/bin/env python3
"""How long do a 1500-B TX batch's checksum-field writes take on their own?

The TX fill patches two 2-B fields per frame in place (2^21 scattered writes at
1500-B stride for 2^20 frames). Inside the receive kernel's read stream they
cost ~60 us over the same kernel writing the checksums as columns. This probe
times the writes alone (torch index_put over a resident 1.5-GB batch: 2-B
writes at frame bytes 24 and 50, and the same as 4 single-byte writes), to
see whether a separate patch pass after the receive pass could be cheaper.
"""
import torch


def timed(fn, reps=20):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    n, stride = 1 << 20, 1500
    buf = torch.randint(0, 256, (n * stride + 64,), dtype=torch.uint8, device=dev)
    base = torch.arange(n, device=dev, dtype=torch.int64) * stride
    w16 = buf.view(torch.int16)
    idx16 = torch.stack([(base + 24) // 2, (base + 50) // 2], 1).flatten()
    v16 = torch.randint(-32768, 32767, (idx16.numel(),), dtype=torch.int16, device=dev)
    idx8 = torch.stack([base + 24, base + 25, base + 50, base + 51], 1).flatten()
    v8 = torch.randint(0, 256, (idx8.numel(),), dtype=torch.uint8, device=dev)
    sums = torch.empty(n, dtype=torch.int64, device=dev)

    def w2():
        w16.index_put_((idx16,), v16)

    def w1():
        buf.index_put_((idx8,), v8)

    def readall():
        torch.sum(buf[: n * stride].view(n, stride)[:, :8].to(torch.int64), dim=1, out=sums)

    print(f"2^20 frames x 2 two-byte field writes (index_put): {timed(w2):8.1f} us")
    print(f"2^20 frames x 4 one-byte writes (index_put):       {timed(w1):8.1f} us")
    print(f"index tensors alone read (2^21 x 8 B):             {timed(lambda: idx16.sum()):8.1f} us")
    print(f"strided 8-B reads of every frame (reference):      {timed(readall):8.1f} us")


if __name__ == "__main__":
    main()
