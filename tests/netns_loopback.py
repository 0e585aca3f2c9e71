#!/usr/bin/env python3
"""configs[0]'s live loopback leg, run inside a fresh user + network namespace.

The parent test starts this script as a new process under
`unshare --user --net --map-root-user` (before this process touches the GPU),
which gives it CAP_NET_RAW / CAP_NET_ADMIN over its own namespace's `lo`. Here:

  1. bring `lo` up (SIOCSIFFLAGS; a new namespace starts with it down);
  2. open the TPACKET_V3 receive ring on lo (libpnet_amd.AfPacket, the
     pnet_datalink Linux receiver, linux.rs:362-403);
  3. send frames over an AF_PACKET socket on lo, as rs_sender.rs:103-105 does
     with tx.send_to: rs_sender's own 64-B frame (rs_sender.rs:25-101, both
     checksums filled) and `--frames` synthetic 64-B UDP/IPv4 frames (1 % with a
     flipped byte);
  4. receive them, as rs_receiver.rs:39-55 does, walking retired blocks;
  5. (--gpu) ship the blocks zero-copy from the mapped ring to the GPU
     (Ring.feed_region) and compare every record with the oracle's; without
     --gpu, the oracle alone parses them (the CPU check of the plumbing).

--pcapdump EXE instead runs examples/pcapdump.c's live mode (`EXE -l lo`) in
the namespace while UDP datagrams go to 127.0.0.1, and reports the lines it
printed for them beside packetdump's expected lines.

Prints one JSON line. Exit 0 = every frame sent was received (each may appear
twice: the outgoing copy and the looped-back one) and, with --gpu, every GPU
record equals the oracle's; exit 3 = the namespace set-up was refused.
"""
import argparse
import fcntl
import json
import os
import socket
import struct
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIOCGIFFLAGS, SIOCSIFFLAGS, IFF_UP = 0x8913, 0x8914, 0x1
ETH_P_ALL = 0x0003


def lo_up():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        r = fcntl.ioctl(s, SIOCGIFFLAGS, struct.pack("16sH14s", b"lo", 0, b""))
        flags = struct.unpack("16sH", r[:18])[1]
        fcntl.ioctl(s, SIOCSIFFLAGS, struct.pack("16sH14s", b"lo", flags | IFF_UP, b""))
    finally:
        s.close()


def pcapdump_live(exe):
    """pcapdump -l lo while 40 datagrams go over lo (tests/test_pcapdump.py)."""
    import subprocess
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    port = rx.getsockname()[1]
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.bind(("127.0.0.1", 0))
    sport = tx.getsockname()[1]
    p = subprocess.Popen([exe, "-l", "lo", "-w", "3000"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(2.0)   # socket open + HIP context before the traffic starts
        if p.poll() is not None:
            print(json.dumps({"early_exit": p.stderr.read()}), flush=True)
            return 1
        want = []
        for i in range(40):
            tx.sendto(b"pnetgpu-live" + bytes(i), ("127.0.0.1", port))
            want.append("[lo]: UDP Packet: 127.0.0.1:%d > 127.0.0.1:%d; length: %d" % (sport, port, 8 + 12 + i))
        try:
            out, err = p.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            out, err = p.communicate()
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
        rx.close()
        tx.close()
    got = sorted({ln for ln in out.splitlines() if ("127.0.0.1:%d" % port) in ln})
    print(json.dumps({"rc": p.returncode, "got": got, "want": sorted(want), "stderr": err[-2000:]}), flush=True)
    return 0 if got == sorted(want) else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20000)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--pcapdump", default=None, help="run pcapdump -l lo (path to the built example)")
    a = ap.parse_args()
    try:
        lo_up()
        tx = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(ETH_P_ALL))
        tx.bind(("lo", 0))
    except OSError as e:
        print(json.dumps({"refused": f"{type(e).__name__}: {e}"}), flush=True)
        return 3
    if a.pcapdump:
        tx.close()
        return pcapdump_live(a.pcapdump)
    import libpnet_amd as lp          # the library only now (no GPU call until --gpu's ring)
    from oracle import coracle        # checker

    rs = lp.synth.make("rs_sender", 1, corrupt_ppm=0)
    w = lp.synth.make("udp64", a.frames, seed=31, corrupt_ppm=10000)
    sent = [bytes(rs.buf[:64])] + [bytes(w.buf[i * 64:(i + 1) * 64]) for i in range(a.frames)]
    afp = lp.AfPacket("lo", block_bytes=1 << 20, n_blocks=32, retire_ms=5)
    t0 = time.perf_counter()
    for f in sent:
        tx.send(f)
    t_send = time.perf_counter() - t0
    want = set(sent)
    seen = set()
    blocks = []                       # (block id, offsets, lengths) of frames we sent
    offs_all, lens_all = [], []
    t0 = time.perf_counter()
    while len(seen) < len(want) and time.perf_counter() - t0 < 20:
        blk = afp.next_block(50)
        if blk is None:
            continue
        k, offs, lens, _ = blk
        keep = [j for j in range(len(offs)) if lens[j] == 64 and bytes(afp.ring[offs[j]:offs[j] + 64]) in want]
        for j in keep:
            seen.add(bytes(afp.ring[offs[j]:offs[j] + 64]))
        if keep:
            offs_all.append(offs[keep])
            lens_all.append(lens[keep])
            blocks.append(k)
        else:
            afp.release(k)
        if len(blocks) >= afp.n_blocks - 2:   # keep ring room: check what we hold, then release
            break
    t_recv = time.perf_counter() - t0
    out = {"sent": len(sent), "distinct_received": len(seen), "send_s": round(t_send, 3),
           "send_mframes_s": round(len(sent) / t_send / 1e6, 3), "recv_s": round(t_recv, 3)}
    offs = np.concatenate(offs_all) if offs_all else np.zeros(0, np.uint64)
    lens = np.concatenate(lens_all) if lens_all else np.zeros(0, np.uint32)
    out["captured"] = int(offs.size)
    # the oracle's records of every captured frame (the receive chain per frame)
    ring_copy = np.array(afp.ring, copy=True)
    rec = coracle.rx_batch(ring_copy, offs.size, offsets=offs, lengths=lens)
    st = rec["status"].astype(np.int64)
    rs_rec = coracle.rx_frame(sent[0])
    out["rs_sender_ip_csum"] = int(rs_rec["ip_csum"])
    out["rs_sender_l4_csum"] = int(rs_rec["l4_csum"])
    out["oracle_l4_bad"] = int(((st & 0x0400) == 0).sum())   # ST_L4_CSUM_OK clear
    ok = len(seen) == len(want)
    if a.gpu and offs.size:
        import torch
        ring = lp.Ring(batch_bytes=8 << 20, batch_frames=1 << 16, copy=True)
        with lp.HostRegistration(afp.ring):
            batches = list(ring.feed_region(afp.ring, offs, lens)) + list(ring.drain())
        ring.close()
        got = {c: np.concatenate([b.records[c] for b in sorted(batches, key=lambda b: b.id)])
               for c in batches[0].records}
        mism = [c for c, v in got.items() if not np.array_equal(v, rec[c])]
        out["gpu_columns_checked"] = len(got)
        out["gpu_mismatched_columns"] = mism
        out["gpu_frames"] = int(sum(b.n for b in batches))
        ok = ok and not mism and out["gpu_frames"] == offs.size
        torch.cuda.synchronize()
    for k in blocks:
        afp.release(k)
    afp.close()
    tx.close()
    out["ok"] = ok
    print(json.dumps(out), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
