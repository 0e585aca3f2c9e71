"""AF_PACKET TPACKET_V3 producer (include/pnetgpu_afpacket.h).

CPU: the block walk over synthetic block images (<linux/if_packet.h> layout,
tests/tpacket.py) incl. malformed ones, and — where this process may open a
packet socket (CAP_NET_RAW; the GPU boxes do not grant it, the build container
does) — a live ring on the loopback interface receiving UDP datagrams sent to
127.0.0.1, parsed by the oracle. GPU: blocks walked and shipped zero-copy
through the ring (Ring.feed_region) give the oracle's records."""
import os
import socket
import struct
import time

import numpy as np
import pytest

import libpnet_amd as lp
from libpnet_amd._lib import PnetGpuError
from oracle import pyoracle
from tests import framegen
from tests.tpacket import BLK_HDR, build_block


@pytest.mark.parametrize("block_bytes,mac_pad", [(1 << 12, 18), (1 << 16, 34), (1 << 20, 18)])
def test_walk_synthetic_blocks(block_bytes, mac_pad):
    rng = np.random.default_rng(block_bytes)
    frames = []
    for f in framegen.random_frames(rng, 2000, max_len=1500):
        try:
            build_block(frames + [f], block_bytes, mac_pad)
        except ValueError:
            break
        frames.append(f)
    blk, starts = build_block(frames, block_bytes, mac_pad)
    o, ln, st = lp.tpacket3_walk(blk, block_offset=7 * block_bytes)
    assert list(o - 7 * block_bytes) == starts
    assert [bytes(blk[a:a + n]) for a, n in zip(o - 7 * block_bytes, ln)] == frames
    assert (st == 1).all()


def test_walk_empty_and_malformed():
    rng = np.random.default_rng(3)
    frames = framegen.random_frames(rng, 20, max_len=200)
    blk, _ = build_block([], 4096)
    assert len(lp.tpacket3_walk(blk)[0]) == 0
    good, _ = build_block(frames, 8192)
    with pytest.raises(PnetGpuError):                       # more packets than cap: EFULL
        lp.tpacket3_walk(good, cap=5)
    bad = good.copy()
    struct.pack_into("<I", bad, 20, 9000)                   # blk_len beyond the block
    with pytest.raises(PnetGpuError):
        lp.tpacket3_walk(bad)
    bad = good.copy()
    struct.pack_into("<I", bad, BLK_HDR, 0)                 # chain ends early
    with pytest.raises(PnetGpuError):
        lp.tpacket3_walk(bad)
    bad = good.copy()
    struct.pack_into("<I", bad, BLK_HDR + 12, 60000)        # snaplen runs past blk_len
    with pytest.raises(PnetGpuError):
        lp.tpacket3_walk(bad)


def test_afpacket_open_validates():
    with pytest.raises((PnetGpuError, PermissionError)):
        lp.AfPacket("no-such-if0")
    with pytest.raises((PnetGpuError, PermissionError)):
        lp.AfPacket("lo", block_bytes=5000)


def test_afpacket_loopback_udp():
    try:
        afp = lp.AfPacket("lo", block_bytes=1 << 16, n_blocks=8, retire_ms=5)
    except PermissionError:
        pytest.skip("no CAP_NET_RAW here")
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    port = rx.getsockname()[1]
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    marker = b"pnetgpu-afp-%d-" % port
    with afp:
        for i in range(300):
            tx.sendto(marker + b"%04d" % i + bytes(i % 40), ("127.0.0.1", port))
        seen = {}
        t0 = time.time()
        while len(seen) < 300 and time.time() - t0 < 10:
            blk = afp.next_block(100)
            if blk is None:
                continue
            k, offs, lens, st = blk
            for o, n, s in zip(offs, lens, st):
                f = bytes(afp.ring[o:o + n])
                j = f.find(marker)
                if j < 0:
                    continue
                r = pyoracle.rx_frame(f)
                assert r["status"] & 3 == pyoracle.ST_L3_IPV4 and r["status"] & 0x1C == pyoracle.ST_L4_UDP
                assert r["status"] & pyoracle.ST_IP_CSUM_OK
                assert r["dst_port"] == port and r["ip_proto"] == 17
                i = int(f[j + len(marker):j + len(marker) + 4])
                assert r["l4_length"] == 8 + len(marker) + 4 + i % 40
                # loopback leaves the UDP checksum to offload: the kernel flags it
                if not r["status"] & pyoracle.ST_L4_CSUM_OK:
                    assert s & lp.afpacket.TP_STATUS_CSUMNOTREADY
                seen[i] = True
            afp.release(k)
        if not seen:
            pytest.skip("no loopback traffic visible to a packet socket here")
        assert len(seen) == 300
        packets, _ = afp.stats()
        assert packets >= 300
    rx.close()
    tx.close()


@pytest.mark.gpu
def test_tpacket3_blocks_through_ring():
    """Four contiguous blocks of a synthetic ring, walked and shipped zero-copy
    (Ring.feed_region from the ring image): records equal the oracle's."""
    from tests.test_gpu_ring import check_batches
    rng = np.random.default_rng(11)
    bb = 1 << 16
    pool = framegen.edge_frames(rng) + framegen.random_frames(rng, 3000, max_len=1500)
    ring_img = np.zeros(4 * bb, np.uint8)
    offs, lens, frames = [], [], []
    p = 0
    for k in range(4):
        chunk = []
        while p < len(pool):
            try:
                build_block(chunk + [pool[p]], bb)
            except ValueError:
                break
            chunk.append(pool[p])
            p += 1
        blk, _ = build_block(chunk, bb)
        ring_img[k * bb:(k + 1) * bb] = blk
        o, ln, _ = lp.tpacket3_walk(ring_img[k * bb:(k + 1) * bb], block_offset=k * bb)
        offs.append(o)
        lens.append(ln)
        frames += chunk
    offs, lens = np.concatenate(offs), np.concatenate(lens)
    ring = lp.Ring(batch_bytes=1 << 17, batch_frames=400)
    with lp.HostRegistration(ring_img):
        out = list(ring.feed_region(ring_img, offs, lens)) + list(ring.drain())
    check_batches(out, frames)


def test_afpacket_fanout_splits_loopback_traffic():
    """Two rings in one PACKET_FANOUT hash group on lo (one per GPU rank in a
    deployment) share the datagrams: together they see every one, each some."""
    try:
        rings = [lp.AfPacket("lo", block_bytes=1 << 16, n_blocks=8, retire_ms=5) for _ in range(2)]
    except PermissionError:
        pytest.skip("no CAP_NET_RAW here")
    group = os.getpid() & 0xFFFF                           # unique per test process
    for r in rings:
        r.fanout(group, "hash")
    # 32 flows: the chance that the hash puts every flow on one ring is 2^-31
    # (with 8 flows it was 1 in 128, an occasional false failure)
    rxs = [socket.socket(socket.AF_INET, socket.SOCK_DGRAM) for _ in range(32)]
    for s_ in rxs:
        s_.bind(("127.0.0.1", 0))
    ports = [s_.getsockname()[1] for s_ in rxs]
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    marker = b"pnetgpu-fanout-%d-" % ports[0]
    for i in range(400):
        tx.sendto(marker + b"%04d" % i, ("127.0.0.1", ports[i % len(ports)]))
    seen = [set(), set()]
    t0 = time.time()
    while len(seen[0] | seen[1]) < 400 and time.time() - t0 < 10:
        for k, r in enumerate(rings):
            blk = r.next_block(20)
            if blk is None:
                continue
            b, offs, lens, _ = blk
            for o, n in zip(offs, lens):
                f = bytes(r.ring[o:o + n])
                j = f.find(marker)
                if j >= 0:
                    seen[k].add(int(f[j + len(marker):j + len(marker) + 4]))
            r.release(b)
    for r in rings:
        r.close()
    for s_ in rxs + [tx]:
        s_.close()
    if not (seen[0] | seen[1]):
        pytest.skip("no loopback traffic visible to a packet socket here")
    assert seen[0] | seen[1] == set(range(400))
    assert seen[0] and seen[1]
