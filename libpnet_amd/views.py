"""pnet_packet-style read-only views over the GPU's per-frame records.

After a batch is processed, a consumer that used pnet_packet's views
(EthernetPacket::new -> Ipv4Packet::new -> UdpPacket::new ..., getters,
payload(); pnet_macros_support/src/packet.rs:19-73, examples/packetdump.rs:120-217)
gets the same answers here without parsing again: `frame_view(records, i, frame)`
returns an object whose constructors answer None exactly where the Rust `new()`
returned None (the record's *_MALFORMED / dispatch bits), whose getters return
the fields the GPU extracted, and whose payload() is a zero-copy memoryview of
the frame bytes at the bounds the GPU computed. Nothing here re-parses a frame.

    b = next(ring.drain())                      # or RxResult.numpy() + the batch bytes
    v = frame_view(b.records, i, b.frames[b.offsets[i]:b.offsets[i] + b.lengths[i]])
    ip = v.ipv4()                               # Ipv4Packet::new(eth.payload()) or None
    if ip and (udp := ip.udp()):                # UdpPacket::new(ip.payload())
        udp.get_source(), udp.payload(), udp.checksum_ok()
"""
import ipaddress

from .engine import DEFS

ST = {k[len("PNET_ST_"):]: v for k, v in DEFS.items() if k.startswith("PNET_ST_")}
_L4 = {ST["L4_UDP"]: "udp", ST["L4_TCP"]: "tcp", ST["L4_ICMP"]: "icmp", ST["L4_ICMPV6"]: "icmpv6"}
_L4_HEADER = {"udp": 8, "tcp": 20, "icmp": 4, "icmpv6": 4}   # payload() starts after the fixed header


def _has(records, name):
    names = getattr(getattr(records, "dtype", None), "names", None)      # a structured record array
    return name in (names if names is not None else records)


def _field(records, name, i):
    if not _has(records, name):
        raise KeyError(f"the batch was processed without the '{name}' column")
    return records[name][i]


class L4View:
    """UdpPacket / TcpPacket / IcmpPacket / Icmpv6Packet over the IP payload."""

    def __init__(self, kind, records, i, frame):
        self.kind, self._r, self._i, self._f = kind, records, i, frame

    def _rec(self, name):
        return _field(self._r, name, self._i)

    def packet(self):
        """The L4 slice (ip.payload()), zero-copy."""
        off, n = int(self._rec("l4_offset")), int(self._rec("l4_length"))
        return memoryview(self._f)[off:off + n]

    def payload(self):
        """Bytes after the fixed header (UDP 8, TCP 20 + options, ICMP 4)."""
        p = self.packet()
        if self.kind == "tcp":
            # the GPU's tcp_data_offset column when the batch computed it
            do = int(self._rec("tcp_data_offset")) if _has(self._r, "tcp_data_offset") else p[12] >> 4
            start = 20 + (do * 4 - 20 if do > 5 else 0)             # tcp.rs:227-236
            return p[start:] if len(p) > start else p[0:0]
        return p[_L4_HEADER[self.kind]:]

    def get_source(self):
        """UDP/TCP source port; for ICMP(v6) the record holds type << 8 | code."""
        return int(self._rec("src_port"))

    def get_destination(self):
        return int(self._rec("dst_port"))

    # ---- header-field columns (ABI v3; KeyError if the batch did not compute them)
    def get_length(self):
        """UdpPacket::get_length (udp.rs:27)."""
        return int(self._rec("udp_length"))

    def get_sequence(self):
        """TcpPacket::get_sequence (tcp.rs:59)."""
        return int(self._rec("tcp_sequence"))

    def get_acknowledgement(self):
        return int(self._rec("tcp_acknowledgement"))

    def get_data_offset(self):
        return int(self._rec("tcp_data_offset"))

    def get_reserved(self):
        return int(self._rec("tcp_reserved"))

    def get_flags(self):
        """TcpPacket::get_flags (tcp.rs:63)."""
        return int(self._rec("tcp_flags"))

    def get_window(self):
        return int(self._rec("tcp_window"))

    def get_urgent_ptr(self):
        return int(self._rec("tcp_urgent_ptr"))

    def get_identifier(self):
        """EchoRequest/EchoReply get_identifier (icmp.rs:228,310): the slice's BE16 at +4."""
        return int(self._rec("dst_port"))

    def get_sequence_number(self):
        """EchoRequest/EchoReply get_sequence_number (icmp.rs:229,311)."""
        return int(self._rec("icmp_sequence"))

    def get_icmp_type(self):
        return int(self._rec("src_port")) >> 8

    def get_icmp_code(self):
        return int(self._rec("src_port")) & 0xFF

    def get_checksum(self):
        """The stored checksum field (big-endian in the frame)."""
        p = self.packet()
        at = {"udp": 6, "tcp": 16, "icmp": 2, "icmpv6": 2}[self.kind]
        return (p[at] << 8) | p[at + 1]

    def computed_checksum(self):
        """udp|tcp::ipv4_checksum / ipv6_checksum, icmp::checksum, icmpv6::checksum;
        None where the reference defines none (ICMPv6 over IPv4)."""
        st = int(self._rec("status"))
        return int(self._rec("l4_csum")) if st & ST["L4_CSUM_DONE"] else None

    def checksum_ok(self):
        st = int(self._rec("status"))
        return bool(st & ST["L4_CSUM_DONE"]) and bool(st & ST["L4_CSUM_OK"])


class IpView:
    """Ipv4Packet / Ipv6Packet over the Ethernet payload."""

    def __init__(self, version, records, i, frame):
        self.version, self._r, self._i, self._f = version, records, i, frame

    def _rec(self, name):
        return _field(self._r, name, self._i)

    def get_source(self):
        if self.version == 4:
            return ipaddress.IPv4Address(int(self._rec("src_ipv4")))
        return ipaddress.IPv6Address(bytes(self._rec("src_ipv6")))

    def get_destination(self):
        if self.version == 4:
            return ipaddress.IPv4Address(int(self._rec("dst_ipv4")))
        return ipaddress.IPv6Address(bytes(self._rec("dst_ipv6")))

    def get_next_level_protocol(self):
        """IPv4 next_level_protocol / IPv6 next_header (after the walk with RX_IPV6_EXT)."""
        return int(self._rec("ip_proto"))

    get_next_header = get_next_level_protocol

    def get_ttl(self):
        return int(self._rec("ttl"))

    get_hop_limit = get_ttl

    # ---- header-field columns (ABI v3; KeyError if the batch did not compute them)
    def get_version(self):
        return int(self._rec("ip_version"))

    def get_header_length(self):
        """Ipv4 IHL (ipv4.rs:141)."""
        return int(self._rec("ip_header_length"))

    def get_dscp(self):
        return int(self._rec("ip_dscp"))

    def get_ecn(self):
        return int(self._rec("ip_ecn"))

    def get_total_length(self):
        return int(self._rec("ip_total_length"))

    def get_identification(self):
        return int(self._rec("ip_identification"))

    def get_flags(self):
        """Ipv4 flags (u3, ipv4.rs:146)."""
        return int(self._rec("ip_flags"))

    def get_fragment_offset(self):
        return int(self._rec("ip_fragment_offset"))

    def get_traffic_class(self):
        """Ipv6 traffic_class (ipv6.rs:24)."""
        return int(self._rec("ip6_traffic_class"))

    def get_flow_label(self):
        return int(self._rec("ip6_flow_label"))

    def get_payload_length(self):
        return int(self._rec("ip6_payload_length"))

    def computed_checksum(self):
        """ipv4::checksum(&ip) (IPv4 only)."""
        return int(self._rec("ip_csum")) if self.version == 4 else None

    def checksum_ok(self):
        return self.version == 4 and bool(int(self._rec("status")) & ST["IP_CSUM_OK"])

    def payload(self):
        """ip.payload(): the L4 slice at the bounds the GPU computed, zero-copy."""
        off, n = int(self._rec("l4_offset")), int(self._rec("l4_length"))
        return memoryview(self._f)[off:off + n]

    def _l4(self, kind):
        st = int(self._rec("status"))
        if _L4.get(st & ST["L4_MASK"]) != kind or st & (ST["L4_MALFORMED"] | ST["FRAGMENT"]):
            return None
        return L4View(kind, self._r, self._i, self._f)

    def udp(self):
        return self._l4("udp")

    def tcp(self):
        return self._l4("tcp")

    def icmp(self):
        return self._l4("icmp")

    def icmpv6(self):
        return self._l4("icmpv6")


class FrameView:
    """EthernetPacket over one processed frame."""

    def __init__(self, records, i, frame):
        self._r, self._i, self._f = records, i, frame

    def _rec(self, name):
        return _field(self._r, name, self._i)

    def valid(self):
        """EthernetPacket::new(frame).is_some() (and the descriptor was in bounds)."""
        return not int(self._rec("status")) & (ST["ETH_MALFORMED"] | ST["DESC_INVALID"])

    def get_ethertype(self):
        """The inner ethertype past any VLAN tags the batch peeled."""
        return int(self._rec("ethertype"))

    def _mac(self, col, at):
        # the GPU's eth_dst / eth_src column (BE-valued u48) when the batch
        # computed it, else the fixed-offset bytes (ethernet.rs:23,25)
        if _has(self._r, col):
            return int(self._rec(col)).to_bytes(6, "big")
        return bytes(self._f[at:at + 6])

    def get_destination(self):
        """MacAddr octets (6 bytes)."""
        return self._mac("eth_dst", 0)

    def get_source(self):
        return self._mac("eth_src", 6)

    def _ip(self, bit, version):
        st = int(self._rec("status"))
        if (st & ST["L3_MASK"]) != bit or st & ST["L3_MALFORMED"]:
            return None
        return IpView(version, self._r, self._i, self._f)

    def ipv4(self):
        """Ipv4Packet::new(eth.payload()): None unless the ethertype is IPv4 and >= 20 B."""
        return self._ip(ST["L3_IPV4"], 4)

    def ipv6(self):
        return self._ip(ST["L3_IPV6"], 6)


def frame_view(records, i, frame):
    """View of frame i: `records` are the batch's columns (RxResult.numpy() or a ring
    Batch's .records; status, plus the columns the getters used read), `frame`
    the frame's bytes (bytes / memoryview / uint8 array)."""
    return FrameView(records, i, frame)
