"""Synthetic TPACKET_V3 block images (the <linux/if_packet.h> layout the kernel
writes into a PACKET_RX_RING): tpacket_block_desc (48 B) then tpacket3_hdr
(48 B) + padding + frame per packet, 16-B aligned, tp_next_offset chained."""
import struct

import numpy as np

BLK_HDR = 48
PKT_HDR = 48


def build_block(frames, block_bytes, mac_pad=18, status=0x1, pkt_status=0x1):
    """One block holding frames (raises if they do not fit). tp_mac = header +
    mac_pad (the kernel leaves room for a sockaddr_ll); tp_net = tp_mac + 14."""
    b = bytearray(block_bytes)
    p = BLK_HDR
    starts = []
    for i, f in enumerate(frames):
        mac = PKT_HDR + mac_pad
        end = p + mac + len(f)
        if end > block_bytes:
            raise ValueError("block full")
        nxt = 0 if i == len(frames) - 1 else ((mac + len(f) + 15) & ~15)
        struct.pack_into("<IIIIIIHH", b, p, nxt, 1700000000 + i, i, len(f), len(f), pkt_status, mac, mac + 14)
        b[p + mac:end] = f
        starts.append(p + mac)
        p += nxt
    blk_len = (p + PKT_HDR + mac_pad + len(frames[-1]) + 15) & ~15 if frames else BLK_HDR
    struct.pack_into("<IIIIII", b, 0, 3, 0, status, len(frames), BLK_HDR, min(blk_len, block_bytes))
    return np.frombuffer(bytes(b), np.uint8), starts
