"""examples/packetdump.rs's output lines, restated in Python for the pcapdump
tests (test infrastructure): the per-frame dispatch and view bounds come from
the oracle's record (oracle/pyoracle.py rx_frame), the text from packetdump.rs's
format strings, the newtypes' derived Debug ("IcmpType(3)", "EtherType(2054)",
...), MacAddr's Display (pnet_base/src/macaddr.rs:101-109) and Rust std's
Ipv4Addr / Ipv6Addr Display. Frames packetdump would panic on (shorter than 14
B: packetdump.rs:291; a 4..7-B ICMP echo: :54,:65) get the lines
examples/pcapdump.c prints instead."""
from oracle import pyoracle as po


def be16(b, i):
    return (b[i] << 8) | b[i + 1]


def mac(b):
    return ":".join(f"{x:02x}" for x in b)


def v4(u):
    return ".".join(str((u >> s) & 255) for s in (24, 16, 8, 0))


def v6(a):
    """Rust's Ipv6Addr Display: ::ffff:a.b.c.d when IPv4-mapped, else the first
    longest run (length >= 2) of zero segments as '::', lowercase hex."""
    s = [be16(a, 2 * i) for i in range(8)]
    if s[:5] == [0] * 5 and s[5] == 0xFFFF:
        return "::ffff:" + ".".join(str(x) for x in a[12:16])
    best = best_len = cur = cur_len = 0
    for i, x in enumerate(s):
        if x == 0:
            if cur_len == 0:
                cur = i
            cur_len += 1
            if cur_len > best_len:
                best, best_len = cur, cur_len
        else:
            cur_len = 0
    h = [f"{x:x}" for x in s]
    if best_len > 1:
        return ":".join(h[:best]) + "::" + ":".join(h[best + best_len:])
    return ":".join(h)


def line(frame, name="pcap", csum=False, l3mode=False):
    r = po.rx_frame(frame, po.RX_L3 if l3mode else 0)
    st = r["status"]
    f = frame
    if st & po.ST_ETH_MALFORMED:
        return f"[{name}]: Malformed Ethernet Frame"
    l3 = st & 3
    if l3 == 0 and l3mode:
        return f"[{name}]: Unknown packet: IP version {f[0] >> 4 if f else 0}; length: {len(f)}"
    if l3 == 0:
        et = r["ethertype"]
        if et == 0x0806:
            if len(f) - 14 < 28:
                return f"[{name}]: Malformed ARP Packet"
            a = f[14:]
            return (f"[{name}]: ARP packet: {mac(f[6:12])}({'.'.join(map(str, a[14:18]))}) > "
                    f"{mac(f[0:6])}({'.'.join(map(str, a[24:28]))}); operation: ArpOperation({be16(a, 6)})")
        return f"[{name}]: Unknown packet: {mac(f[6:12])} > {mac(f[0:6])}; ethertype: EtherType({et}) length: {len(f)}"
    ipname = "IPv4" if l3 == 1 else "IPv6"
    if st & po.ST_L3_MALFORMED:
        return f"[{name}]: Malformed {ipname} Packet"
    if l3 == 1:
        src, dst = v4(r["src_ipv4"]), v4(r["dst_ipv4"])
    else:
        src, dst = v6(r["src_ipv6"]), v6(r["dst_ipv6"])
    sfx = ""
    if csum:
        if l3 == 1:
            sfx += "; ip checksum " + ("ok" if st & po.ST_IP_CSUM_OK else "bad")
        if st & po.ST_L4_CSUM_DONE:
            sfx += "; l4 checksum " + ("ok" if st & po.ST_L4_CSUM_OK else "bad")
    l4 = f[r["l4_offset"]:r["l4_offset"] + r["l4_length"]]
    bad = bool(st & po.ST_L4_MALFORMED)
    kind = st & 0x1C
    if kind == po.ST_L4_UDP:
        if bad:
            return f"[{name}]: Malformed UDP Packet"
        return f"[{name}]: UDP Packet: {src}:{be16(l4, 0)} > {dst}:{be16(l4, 2)}; length: {be16(l4, 4)}{sfx}"
    if kind == po.ST_L4_TCP:
        if bad:
            return f"[{name}]: Malformed TCP Packet"
        return f"[{name}]: TCP Packet: {src}:{be16(l4, 0)} > {dst}:{be16(l4, 2)}; length: {len(l4)}{sfx}"
    if kind == po.ST_L4_ICMP:
        if bad or (l4[0] in (0, 8) and len(l4) < 8):
            return f"[{name}]: Malformed ICMP Packet"
        if l4[0] in (0, 8):
            what = "request" if l4[0] == 8 else "reply"
            return f"[{name}]: ICMP echo {what} {src} -> {dst} (seq={be16(l4, 6)}, id={be16(l4, 4)}){sfx}"
        return f"[{name}]: ICMP packet {src} -> {dst} (type=IcmpType({l4[0]})){sfx}"
    if kind == po.ST_L4_ICMPV6:
        if bad:
            return f"[{name}]: Malformed ICMPv6 Packet"
        return f"[{name}]: ICMPv6 packet {src} -> {dst} (type=Icmpv6Type({l4[0]})){sfx}"
    return (f"[{name}]: Unknown {ipname} packet: {src} > {dst}; protocol: IpNextHeaderProtocol({r['ip_proto']}) "
            f"length: {len(l4)}{sfx}")
