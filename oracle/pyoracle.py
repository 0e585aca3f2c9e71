"""Independent pure-Python restatement of the receive path (small cases only).

TEST INFRASTRUCTURE ONLY. A second, separately written restatement of the
reference semantics used to cross-check the C oracle (oracle/pnet_oracle.c) on
random and edge-case frames. Written from the reference, not from the C file:

  sum_be_words      pnet_packet/src/util.rs:158-181
  finalize          pnet_packet/src/util.rs:84-89
  checksum          pnet_packet/src/util.rs:76-82
  ipv4/ipv6_checksum pnet_packet/src/util.rs:92-154
  receive dispatch  examples/packetdump.rs:120-217 + the #[packet] layouts
"""

ST_L3_IPV4 = 0x0001
ST_L3_IPV6 = 0x0002
ST_L4_UDP = 1 << 2
ST_L4_TCP = 2 << 2
ST_L4_ICMP = 3 << 2
ST_L4_ICMPV6 = 4 << 2
ST_ETH_MALFORMED = 0x0020
ST_L3_MALFORMED = 0x0040
ST_L4_MALFORMED = 0x0080
ST_IP_CSUM_OK = 0x0100
ST_L4_CSUM_DONE = 0x0200
ST_L4_CSUM_OK = 0x0400
ST_UNKNOWN_ETHERTYPE = 0x0800
ST_UNKNOWN_PROTO = 0x1000
ST_VLAN = 0x2000
ST_FRAGMENT = 0x4000
ST_DESC_INVALID = 0x8000
RX_VLAN, RX_IPV6_EXT, RX_L3 = 0x1, 0x2, 0x4

# Header-field getters, restated from the #[packet] declarations: each layout
# lists (getter, bit width) in declaration order, and a generated getter reads
# its width of bits at the running bit offset, most significant bit first
# (pnet_macros/src/decorator.rs:1563-1670). Names starting with "_" are fields
# this record does not keep (or keeps under a dispatch name).
ETHERNET = (("eth_dst", 48), ("eth_src", 48), ("_ethertype", 16))                        # ethernet.rs:20-30
IPV4 = (("ip_version", 4), ("ip_header_length", 4), ("ip_dscp", 6), ("ip_ecn", 2),       # ipv4.rs:138-161
        ("ip_total_length", 16), ("ip_identification", 16), ("ip_flags", 3), ("ip_fragment_offset", 13))
IPV6 = (("ip_version", 4), ("ip6_traffic_class", 8), ("ip6_flow_label", 20),             # ipv6.rs:21-37
        ("ip6_payload_length", 16))
UDP = (("_source", 16), ("_destination", 16), ("udp_length", 16))                        # udp.rs:23-31
TCP = (("_source", 16), ("_destination", 16), ("tcp_sequence", 32), ("tcp_acknowledgement", 32),  # tcp.rs:55-71
       ("tcp_data_offset", 4), ("tcp_reserved", 4), ("tcp_flags", 8), ("tcp_window", 16), ("_checksum", 16),
       ("tcp_urgent_ptr", 16))
ECHO = (("_icmp_type", 8), ("_icmp_code", 8), ("_checksum", 16), ("_identifier", 16),     # icmp.rs:221-232
        ("icmp_sequence", 16))

HEADER_FIELDS = tuple(dict.fromkeys(n for lay in (ETHERNET, IPV4, IPV6, UDP, TCP, ECHO) for n, _ in lay
                                    if not n.startswith("_")))

FIELDS = ("status", "ip_csum", "l4_csum", "ethertype", "ip_proto", "ttl", "l4_offset",
          "l4_length", "src_port", "dst_port", "src_ipv4", "dst_ipv4", "src_ipv6", "dst_ipv6",
          "vlan_tci", "l3_offset") + HEADER_FIELDS


def getters(buf, layout):
    """Values of a view's generated getters over the first bytes of buf."""
    bits = sum(w for _, w in layout)
    nbytes = (bits + 7) // 8
    v = int.from_bytes(bytes(buf[:nbytes]), "big")
    out, at = {}, 0
    for name, w in layout:
        if not name.startswith("_"):
            out[name] = (v >> (8 * nbytes - at - w)) & ((1 << w) - 1)
        at += w
    return out


def sum_be_words(d, skip):
    d = bytes(d)
    if not d:
        return 0
    words = [(d[2 * i] << 8) | d[2 * i + 1] for i in range(len(d) // 2)]
    s = sum(w for i, w in enumerate(words) if i != skip)
    if len(d) % 2 and len(d) // 2 != skip:
        s += d[-1] << 8
    return s & 0xFFFFFFFF


def finalize(s):
    while s >> 16:
        s = (s >> 16) + (s & 0xFFFF)
    return (~s) & 0xFFFF


def checksum(d, skip):
    return 0 if len(d) == 0 else finalize(sum_be_words(d, skip))


def _segsum(addr):
    a = bytes(addr)
    return sum((a[i] << 8) | a[i + 1] for i in range(0, len(a), 2))


def ipv4_checksum(d, skip, extra, src, dst, proto):
    s = _segsum(src) + _segsum(dst) + proto + len(d) + len(extra)
    s += sum_be_words(d, skip) + sum_be_words(extra, len(extra) // 2)
    return finalize(s & 0xFFFFFFFF)


ipv6_checksum = ipv4_checksum  # identical arithmetic over 8 segments per address


def _be16(b, i):
    return (b[i] << 8) | b[i + 1]


def rx_frame(frame, flags=0):
    f = bytes(frame)
    r = dict.fromkeys(FIELDS, 0)
    r["src_ipv6"] = bytes(16)
    r["dst_ipv6"] = bytes(16)
    st = 0
    if flags & RX_L3:                        # pnet_transport Layer3: IP header at byte 0
        ver = f[0] >> 4 if f else 0
        et = {4: 0x0800, 6: 0x86DD}.get(ver, 0)
        l3 = 0
    else:
        if len(f) < 14:
            r["status"] = ST_ETH_MALFORMED
            return r
        et = _be16(f, 12)
        l3 = 14
        r.update(getters(f, ETHERNET))
    if flags & RX_VLAN and not flags & RX_L3:   # vlan.rs:62-72; TPIDs ethernet.rs:102,104,112
        for k in range(2):
            if et not in (0x8100, 0x88A8, 0x9100):
                break
            st |= ST_VLAN
            if len(f) < l3 + 4:
                r["ethertype"], r["status"] = et, st | ST_L3_MALFORMED
                return r
            if k == 0:
                r["vlan_tci"] = _be16(f, l3)
            et = _be16(f, l3 + 2)
            l3 += 4
    r["ethertype"] = et
    r["l3_offset"] = l3
    ep = f[l3:]
    if et == 0x0800:
        st |= ST_L3_IPV4
        if len(ep) < 20:
            r["status"] = st | ST_L3_MALFORMED
            return r
        r.update(getters(ep, IPV4))
        ihl = ep[0] & 15
        hl = min(max(ihl * 4, 20), len(ep))
        r["ip_csum"] = checksum(ep[:hl], 5)
        if r["ip_csum"] == _be16(ep, 10):
            st |= ST_IP_CSUM_OK
        r["ttl"], r["ip_proto"] = ep[8], ep[9]
        r["src_ipv4"] = int.from_bytes(ep[12:16], "big")
        r["dst_ipv4"] = int.from_bytes(ep[16:20], "big")
        start = 20 + max(ihl * 4 - 20, 0)
        plen = max(_be16(ep, 2) - ihl * 4, 0)
        l4 = b""
        if len(ep) > start:
            l4 = ep[start:min(start + plen, len(ep))]
            r["l4_offset"], r["l4_length"] = l3 + start, len(l4)
        src, dst, proto, v6 = ep[12:16], ep[16:20], ep[9], False
    elif et == 0x86DD:
        st |= ST_L3_IPV6
        if len(ep) < 40:
            r["status"] = st | ST_L3_MALFORMED
            return r
        r.update(getters(ep, IPV6))
        r["ip_proto"], r["ttl"] = ep[6], ep[7]
        r["src_ipv6"], r["dst_ipv6"] = ep[8:24], ep[24:40]
        pl = ep[40:min(40 + _be16(ep, 4), len(ep))] if len(ep) > 40 else b""
        proto, pos = ep[6], 0
        if flags & RX_IPV6_EXT:              # ipv6.rs:39-137
            for _ in range(4):
                if proto in (0, 60, 43):
                    if len(pl) - pos < (4 if proto == 43 else 2) or pl[pos + 1] * 8 + 8 > len(pl) - pos:
                        r["ip_proto"], r["status"] = proto, st | ST_L4_MALFORMED
                        return r
                    proto, pos = pl[pos], pos + pl[pos + 1] * 8 + 8
                elif proto == 44:
                    if len(pl) - pos < 8:
                        r["ip_proto"], r["status"] = proto, st | ST_L4_MALFORMED
                        return r
                    fo = _be16(pl, pos + 2)
                    proto, pos = pl[pos], pos + 8
                    if fo & 0xFFFC:
                        r["ip_proto"] = proto
                        if len(pl) > pos:
                            r["l4_offset"], r["l4_length"] = l3 + 40 + pos, len(pl) - pos
                        r["status"] = st | ST_FRAGMENT
                        return r
                else:
                    break
            r["ip_proto"] = proto
        l4 = pl[pos:]
        if l4:
            r["l4_offset"], r["l4_length"] = l3 + 40 + pos, len(l4)
        src, dst, v6 = ep[8:24], ep[24:40], True
    else:
        r["status"] = st | ST_UNKNOWN_ETHERTYPE
        return r

    table = {17: (ST_L4_UDP, 8, 3, 6), 6: (ST_L4_TCP, 20, 8, 16),
             1: (ST_L4_ICMP, 4, 1, 2), 58: (ST_L4_ICMPV6, 4, 1, 2)}
    if proto not in table:
        r["status"] = st | ST_UNKNOWN_PROTO
        return r
    kind, minlen, skip, csum_at = table[proto]
    st |= kind
    if len(l4) < minlen:
        r["status"] = st | ST_L4_MALFORMED
        return r
    r["src_port"] = _be16(l4, 0)
    if proto in (17, 6):
        r["dst_port"] = _be16(l4, 2)
        r.update(getters(l4, UDP if proto == 17 else TCP))
    else:
        r["dst_port"] = _be16(l4, 4) if len(l4) >= 8 else 0
        # EchoRequest/EchoReply view (minimum 8 bytes) for the echo types only:
        # ICMP 0/8 (packetdump.rs:52-75), ICMPv6 128/129 (icmpv6.rs:135-137)
        if len(l4) >= 8 and l4[0] in ((0, 8) if proto == 1 else (128, 129)):
            r.update(getters(l4, ECHO))
    c = None
    if proto == 1:
        c = checksum(l4, 1)
    elif proto == 58:
        if v6:
            c = ipv6_checksum(l4, 1, b"", src, dst, 58)
    else:
        c = ipv4_checksum(l4, skip, b"", src, dst, proto)
    if c is not None:
        r["l4_csum"] = c
        st |= ST_L4_CSUM_DONE
        if c == _be16(l4, csum_at):
            st |= ST_L4_CSUM_OK
    r["status"] = st
    return r
