"""Seeded test-frame factory: well-formed, corrupted and malformed Ethernet frames.

Builds frames by the reference's own construction rules (benches/rs_sender.rs,
src/pnettest.rs builders) with random field values, then perturbs them to hit
every edge the reference tests: IHL 0-15,
total_length below/above the buffer, odd L4 lengths, TCP data offsets 0-15,
short frames, unknown ethertypes/protocols, checksum zero and flipped bytes.
Checksums of well-formed frames are filled in with the pure-Python
restatement (oracle/pyoracle.py) — construction only, never the checker.
"""
import numpy as np

from oracle import pyoracle as po


def _set16(b, i, v):
    b[i] = (v >> 8) & 0xFF
    b[i + 1] = v & 0xFF


def build_frame(rng, kind, l4_len, ihl=5, vlan=False):
    """A valid frame: kind in {'udp','tcp','icmp','udp6','tcp6','icmp6','icmp_over6'}."""
    v6 = kind in ("udp6", "tcp6", "icmp6", "icmp_over6")
    proto = {"udp": 17, "tcp": 6, "icmp": 1, "udp6": 17, "tcp6": 6, "icmp6": 58,
             "icmp_over6": 1}[kind]
    iphl = 40 if v6 else ihl * 4
    f = bytearray(14 + iphl + l4_len)
    f[0:12] = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
    _set16(f, 12, 0x86DD if v6 else 0x0800)
    ip = 14
    if v6:
        f[ip] = 0x60 | int(rng.integers(0, 16))
        f[ip + 1:ip + 4] = rng.integers(0, 256, 3, dtype=np.uint8).tobytes()
        _set16(f, ip + 4, l4_len)
        f[ip + 6] = proto
        f[ip + 7] = int(rng.integers(1, 256))
        f[ip + 8:ip + 40] = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
    else:
        f[ip] = 0x40 | ihl
        f[ip + 1] = int(rng.integers(0, 256))
        _set16(f, ip + 2, iphl + l4_len)
        f[ip + 4:ip + 8] = rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        f[ip + 8] = int(rng.integers(1, 256))
        f[ip + 9] = proto
        f[ip + 12:ip + 20] = rng.integers(0, 256, 8, dtype=np.uint8).tobytes()
        f[ip + 20:ip + iphl] = rng.integers(0, 256, iphl - 20, dtype=np.uint8).tobytes()
        _set16(f, ip + 10, po.checksum(bytes(f[ip:ip + iphl]), 5))
    l4 = 14 + iphl
    f[l4:] = rng.integers(0, 256, l4_len, dtype=np.uint8).tobytes()
    if proto == 6 and l4_len >= 20:
        f[l4 + 12] = (5 << 4) | (f[l4 + 12] & 0x0F)
    seg = bytes(f[l4:])
    if v6:
        src, dst = bytes(f[ip + 8:ip + 24]), bytes(f[ip + 24:ip + 40])
    else:
        src, dst = bytes(f[ip + 12:ip + 16]), bytes(f[ip + 16:ip + 20])
    if proto == 17 and l4_len >= 8:
        _set16(f, l4 + 4, l4_len)
        seg = bytes(f[l4:])
        _set16(f, l4 + 6, po.ipv4_checksum(seg, 3, b"", src, dst, 17))
    elif proto == 6 and l4_len >= 20:
        _set16(f, l4 + 16, po.ipv4_checksum(seg, 8, b"", src, dst, 6))
    elif proto == 1 and l4_len >= 4:
        _set16(f, l4 + 2, po.checksum(seg, 1))
    elif proto == 58 and l4_len >= 4:
        _set16(f, l4 + 2, po.ipv6_checksum(seg, 1, b"", src, dst, 58))
    return bytes(f)


def edge_frames(rng):
    """A fixed list of edge-case frames (deterministic for a given rng seed)."""
    out = []
    # short frames: 0..70 bytes of random data, and the prefixes of a valid frame
    for n in range(0, 71):
        out.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    base = build_frame(rng, "tcp", 40)
    for n in range(0, len(base) + 1, 3):
        out.append(base[:n])
    base6 = build_frame(rng, "udp6", 21)
    for n in range(0, len(base6) + 1, 5):
        out.append(base6[:n])
    # IHL 0..15 with various total_length (below, equal, above the buffer)
    for ihl in range(16):
        for tl in (0, 1, 19, 20, 21, ihl * 4, ihl * 4 + 7, 33, 60, 64, 500, 65535):
            for proto in (17, 6, 1, 58, 253):
                f = bytearray(build_frame(rng, "udp", 30, ihl=max(ihl, 5)))
                f[14] = (f[14] & 0xF0) | ihl
                _set16(f, 16, tl)
                f[23] = proto
                out.append(bytes(f))
    # TCP data offsets 0..15, odd lengths
    for do in range(16):
        for l4 in (19, 20, 21, 33, 64):
            f = bytearray(build_frame(rng, "tcp", l4))
            if len(f) > 14 + 20 + 12:
                f[14 + 20 + 12] = (do << 4) | (f[14 + 20 + 12] & 15)
            out.append(bytes(f))
    # odd / even L4 lengths for every kind, valid checksums
    for kind in ("udp", "tcp", "icmp", "udp6", "tcp6", "icmp6", "icmp_over6"):
        for l4 in (0, 1, 3, 4, 7, 8, 9, 13, 19, 20, 21, 64, 65, 100, 255):
            out.append(build_frame(rng, kind, l4))
    # UDP checksum field zero (not special-cased by the reference)
    f = bytearray(build_frame(rng, "udp", 13))
    f[14 + 20 + 6] = f[14 + 20 + 7] = 0
    out.append(bytes(f))
    # all-zero / all-0xff bodies with valid ethertypes
    for et in (0x0800, 0x86DD, 0x0806, 0x8100):
        for fill in (0, 0xFF):
            b = bytearray([fill]) * 80
            _set16(b, 12, et)
            out.append(bytes(b))
    # ICMPv6 over IPv4 (no checksum defined), ICMP over IPv6
    f = bytearray(build_frame(rng, "icmp", 12))
    f[23] = 58
    out.append(bytes(f))
    return out


def random_frames(rng, n, min_len=0, max_len=1600):
    """A mix of valid, corrupted, truncated and padded frames."""
    kinds = ("udp", "tcp", "icmp", "udp6", "tcp6", "icmp6", "icmp_over6")
    out = []
    for _ in range(n):
        r = rng.random()
        kind = kinds[int(rng.integers(0, len(kinds)))]
        l4 = int(rng.integers(0, max(1, max_len - 60)))
        f = bytearray(build_frame(rng, kind, l4, ihl=int(rng.integers(5, 16))))
        if r < 0.15 and len(f):          # flip one byte
            i = int(rng.integers(0, len(f)))
            f[i] ^= int(rng.integers(1, 256))
        elif r < 0.25:                   # truncate
            f = f[:int(rng.integers(0, len(f) + 1))]
        elif r < 0.35:                   # Ethernet padding after the IP datagram
            f += rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
        elif r < 0.40:                   # random IHL / total_length
            if len(f) > 18 and f[12:14] == b"\x08\x00":
                f[14] = (f[14] & 0xF0) | int(rng.integers(0, 16))
                _set16(f, 16, int(rng.integers(0, 2000)))
        elif r < 0.43:                   # garbage
            f = bytearray(rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8))
        f = f[:max_len] if len(f) > max_len else f
        if len(f) < min_len:
            f += bytes(min_len - len(f))
        out.append(bytes(f))
    return out


def pack(frames, align=1, gap=0, rng=None):
    """Pack frames into one buffer; returns (buf uint8, offsets u64, lengths u32).

    align: each frame starts at a multiple of `align`; gap: random 0..gap extra
    bytes between frames (exercises arbitrary start alignment)."""
    offs, lens, parts, pos = [], [], [], 0
    for f in frames:
        pad = (-pos) % align
        if gap and rng is not None:
            pad += int(rng.integers(0, gap + 1))
        if pad:
            parts.append(bytes(pad))
            pos += pad
        offs.append(pos)
        lens.append(len(f))
        parts.append(f)
        pos += len(f)
    parts.append(bytes((-pos) % 16 + 16))  # readable tail up to a 16-B multiple
    buf = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return buf, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint32)


# ---- opt-in extensions: VLAN tags and IPv6 extension headers ----------------

def add_vlan(frame, tags):
    """Insert VLAN tags (list of (tpid, tci)) after the MAC addresses."""
    f = bytes(frame)
    if len(f) < 14:
        return f
    out = bytearray(f[:12])
    for tpid, tci in tags:
        out += tpid.to_bytes(2, "big") + tci.to_bytes(2, "big")
    out += f[12:]
    # the tags' inner ethertypes chain: tag k's "ethertype" field is the next TPID / the real one
    pos = 12
    tpids = [t for t, _ in tags] + [int.from_bytes(f[12:14], "big")]
    for k in range(len(tags)):
        out[pos:pos + 2] = tpids[k].to_bytes(2, "big")
        out[pos + 4:pos + 6] = tpids[k + 1].to_bytes(2, "big")
        pos += 4
    return bytes(out)


def ipv6_with_ext(rng, exts, l4_kind, l4_len, frag_offset=0):
    """An Eth/IPv6 frame whose payload is a chain of extension headers then L4.
    exts: list of header type ids (0, 43, 44, 60); checksums are valid for the
    final L4 (pseudo-header = base addresses + L4 slice length)."""
    proto = {"udp": 17, "tcp": 6, "icmp6": 58, "icmp": 1, "none": 59}[l4_kind]
    chain = bytearray()
    types = list(exts) + [proto]
    for k, t in enumerate(exts):
        nxt = types[k + 1]
        if t == 44:
            fo = (frag_offset << 3) & 0xFFF8
            chain += bytes([nxt, 0]) + fo.to_bytes(2, "big") + rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
        else:
            hel = int(rng.integers(0, 4))
            body = rng.integers(0, 256, hel * 8 + 6, dtype=np.uint8).tobytes()
            if t == 43:
                body = bytes([int(rng.integers(0, 4)), int(rng.integers(0, 3))]) + body[2:]
            chain += bytes([nxt, hel]) + body
    base = bytearray(build_frame(rng, "udp6", 8))[:54]
    base[20] = types[0] if exts else proto
    l4 = bytearray(rng.integers(0, 256, l4_len, dtype=np.uint8).tobytes())
    src, dst = bytes(base[22:38]), bytes(base[38:54])
    if proto == 17 and l4_len >= 8:
        _set16(l4, 4, l4_len)
        _set16(l4, 6, 0)
        _set16(l4, 6, po.ipv6_checksum(bytes(l4), 3, b"", src, dst, 17))
    elif proto == 6 and l4_len >= 20:
        l4[12] = 5 << 4
        _set16(l4, 16, 0)
        _set16(l4, 16, po.ipv6_checksum(bytes(l4), 8, b"", src, dst, 6))
    elif proto == 58 and l4_len >= 4:
        _set16(l4, 2, 0)
        _set16(l4, 2, po.ipv6_checksum(bytes(l4), 1, b"", src, dst, 58))
    elif proto == 1 and l4_len >= 4:
        _set16(l4, 2, 0)
        _set16(l4, 2, po.checksum(bytes(l4), 1))
    payload = bytes(chain) + bytes(l4)
    _set16(base, 18, len(payload))
    return bytes(base) + payload


def extension_frames(rng):
    """VLAN / QinQ / IPv6-extension frames incl. truncations and long chains."""
    out = []
    kinds = ("udp", "tcp", "icmp", "udp6", "tcp6", "icmp6")
    tag_sets = ([], [(0x8100, 0x0064)], [(0x88A8, 0x2001), (0x8100, 0xE00A)], [(0x9100, 5), (0x9100, 6)],
                [(0x8100, 1), (0x8100, 2), (0x8100, 3)])
    for tags in tag_sets:
        for k in kinds:
            for l4 in (0, 4, 8, 13, 20, 33, 200):
                out.append(add_vlan(build_frame(rng, k, l4, ihl=int(rng.integers(5, 16))), tags))
    # truncated tags
    f = add_vlan(build_frame(rng, "udp", 20), [(0x8100, 7), (0x8100, 8)])
    for n in range(12, 26):
        out.append(f[:n])
    # IPv6 extension chains
    chains = ([], [0], [60], [43], [44], [0, 60], [0, 43, 44], [0, 60, 43, 44], [0, 60, 43, 60, 44], [44, 44])
    for exts in chains:
        for l4k in ("udp", "tcp", "icmp6", "icmp", "none"):
            for l4 in (0, 3, 8, 21, 64, 700):
                out.append(ipv6_with_ext(rng, exts, l4k, l4))
    for off in (1, 100, 8191):
        out.append(ipv6_with_ext(rng, [0, 44], "udp", 40, frag_offset=off))
    # long chains: the L4 header lands past the 128-B window
    for _ in range(20):
        exts = [int(x) for x in rng.choice([0, 43, 60], size=4)]
        out.append(add_vlan(ipv6_with_ext(rng, exts, "tcp", int(rng.integers(20, 400))),
                            [(0x8100, 9)] if rng.random() < 0.5 else []))
    # truncated extension headers
    g = ipv6_with_ext(rng, [0, 43, 60], "udp", 30)
    for n in range(54, len(g) + 1, 3):
        h = bytearray(g[:n])
        out.append(bytes(h))
    return out


def icmp_type_frames(rng):
    """ICMP over IPv4 and ICMPv6 over IPv6 frames of every echo / non-echo type the
    echo-view gate distinguishes (icmp_sequence is the EchoRequest/EchoReply
    get_sequence_number for ICMP 0/8 and ICMPv6 128/129 only, packetdump.rs:52-75,
    icmpv6.rs:135-137), with 4-, 7-, 8- and 24-B slices. Returns (frames, echo?)."""
    frames, echo = [], []
    for kind, types, ok in (("icmp", (0, 3, 5, 8, 11, 128), (0, 8)), ("icmp6", (0, 1, 8, 128, 129, 135), (128, 129))):
        for t in types:
            for l4_len in (4, 7, 8, 24):
                f = bytearray(build_frame(rng, kind, l4_len))
                l4 = len(f) - l4_len
                f[l4] = t
                f[l4 + 2:l4 + 4] = b"\0\0"
                seg = bytes(f[l4:])
                if kind == "icmp":
                    c = po.checksum(seg, 1)
                else:
                    c = po.ipv6_checksum(seg, 1, b"", bytes(f[22:38]), bytes(f[38:54]), 58)
                _set16(f, l4 + 2, c)
                frames.append(bytes(f))
                echo.append(t in ok and l4_len >= 8)
    return frames, echo
