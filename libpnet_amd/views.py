"""pnet_packet-style read-only views over the GPU's per-frame records.

After a batch is processed, a consumer that used pnet_packet's views
(EthernetPacket::new -> Ipv4Packet::new -> UdpPacket::new ..., getters,
payload(); pnet_macros_support/src/packet.rs:19-73, examples/packetdump.rs:120-217)
gets the same answers here without parsing again: `frame_view(records, i, frame)`
returns an object whose constructors answer None exactly where the Rust `new()`
returned None (the record's *_MALFORMED / dispatch bits), whose getters return
the fields the GPU extracted, and whose payload() is a zero-copy memoryview of
the frame bytes at the bounds the GPU computed. Nothing here re-parses a frame.

The rest of the trait surface (pnet_macros_support/src/packet.rs:19-89):
`packet()` / `payload()` (Packet), `packet_mut()` / `payload_mut()` /
`clone_from()` (MutablePacket: writable views when the frame buffer is
writable — edit, then recompute the checksums of the whole batch with
tx_fill_checksums), the generated `minimum_packet_size()` and
`to_immutable()` (decorator.rs:589-632), `packet_size()`
(PacketSize, the generated header + variable-field sizes) and `from_packet()`
(FromPacket: an owned dict of every field). IPv4 and TCP options are decoded
from the option bytes between the fixed header and the bounds the record
gives, by the generated Ipv4OptionIterable / TcpOptionIterable rules
(`get_options_iter()`, ipv4.rs:156-157,258-290; tcp.rs:68,107-210).

    b = next(ring.drain())                      # or RxResult.numpy() + the batch bytes
    v = frame_view(b.records, i, b.frames[b.offsets[i]:b.offsets[i] + b.lengths[i]])
    ip = v.ipv4()                               # Ipv4Packet::new(eth.payload()) or None
    if ip and (udp := ip.udp()):                # UdpPacket::new(ip.payload())
        udp.get_source(), udp.payload(), udp.checksum_ok()
"""
import copy
import ipaddress
from dataclasses import dataclass

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


def _writable(buf, what):
    mv = memoryview(buf)
    if mv.readonly:
        raise TypeError(f"{what}: the frame buffer is read-only (pass a bytearray / numpy array to mutate)")
    return mv


def _be16(b, at):
    return (b[at] << 8) | b[at + 1]


#: minimum_packet_size() of each view: the byte size of its fixed fields, the
#: bound every generated new() checks (pnet_macros/src/decorator.rs:589-600,623-629)
MINIMUM_PACKET_SIZE = {"ethernet": 14, "ipv4": 20, "ipv6": 40, "udp": 8, "tcp": 20, "icmp": 4, "icmpv6": 4,
                       "echo_request": 8, "echo_reply": 8, "destination_unreachable": 8, "time_exceeded": 8}


class _PacketTraits:
    """The generated inherent methods and MutablePacket defaults every view shares
    (pnet_macros/src/decorator.rs:589-632, pnet_macros_support/src/packet.rs:61-72)."""

    def to_immutable(self):
        """MutableXxxPacket::to_immutable: the same view over a read-only buffer
        (packet_mut / payload_mut / clone_from then raise)."""
        v = copy.copy(self)
        v._f = memoryview(self._f).toreadonly()
        return v

    consume_to_immutable = to_immutable

    def clone_from(self, other):
        """MutablePacket::clone_from: copy other.packet() (another view, or bytes)
        over the start of this view's packet_mut(). Like the reference, asserts
        that this packet is at least as long as the other."""
        src = bytes(other.packet() if hasattr(other, "packet") else other)
        assert len(self.packet()) >= len(src), "clone_from: the destination packet is shorter than the source"
        self.packet_mut()[:len(src)] = src


@dataclass(frozen=True)
class Ipv4Option:
    """Ipv4Option (ipv4.rs:258-290): copied u1, class u2, number u5, the optional
    length byte (empty for EOL 0 / NOP 1) and the data (length - 2 bytes, bounded
    by the option buffer)."""
    copied: int
    class_: int
    number: int
    length: bytes
    data: bytes


@dataclass(frozen=True)
class TcpOption:
    """TcpOption (tcp.rs:107-116): number u8, the optional length byte (empty for
    EOL 0 / NOP 1) and the data (length - 2 bytes when length >= 2, bounded by the
    option buffer, tcp.rs:198-210)."""
    number: int
    length: bytes
    data: bytes


def _option_iter(buf, tcp):
    """The generated {Ipv4Option,TcpOption}Iterable (pnet_macros decorator.rs:772-810):
    while bytes remain, XxxOptionPacket::new(buf) (1-B minimum), then advance by
    min(packet_size, remaining), packet_size = 1 + len(length) + len(data)."""
    buf = bytes(buf)
    while buf:
        first = buf[0]
        number = first if tcp else first & 0x1F
        ll = 0 if number in (0, 1) else 1                 # ipv4.rs:276-282, tcp.rs:191-198
        length = buf[1:1 + ll]                            # get_length(): bounded by the buffer
        if tcp:
            plen = length[0] - 2 if length and length[0] >= 2 else 0     # tcp.rs:206-210
        else:
            plen = max(length[0] - 2, 0) if length else 0                # ipv4.rs:285-290
        lo = min(1 + ll, len(buf))
        data = buf[lo:max(min(1 + ll + plen, len(buf)), lo)]
        yield (TcpOption(number, length, data) if tcp else
               Ipv4Option(first >> 7, (first >> 5) & 3, number, length, data))
        buf = buf[min(1 + ll + plen, len(buf)):]


class L4View(_PacketTraits):
    """UdpPacket / TcpPacket / IcmpPacket / Icmpv6Packet over the IP payload."""

    def __init__(self, kind, records, i, frame):
        self.kind, self._r, self._i, self._f = kind, records, i, frame

    def minimum_packet_size(self):
        """UdpPacket 8, TcpPacket 20, IcmpPacket / Icmpv6Packet 4 (their new() bounds)."""
        return MINIMUM_PACKET_SIZE[self.kind]

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

    def _tcp_data_offset(self, p):
        return int(self._rec("tcp_data_offset")) if _has(self._r, "tcp_data_offset") else p[12] >> 4

    def _bounds(self):
        return int(self._rec("l4_offset")), int(self._rec("l4_length"))

    def packet_mut(self):
        """MutablePacket::packet_mut: the L4 slice, writable (the frame buffer must be)."""
        off, n = self._bounds()
        return _writable(self._f, "packet_mut")[off:off + n]

    def payload_mut(self):
        """MutablePacket::payload_mut: payload() over the writable frame buffer."""
        off, n = self._bounds()
        start = len(self.packet()) - len(self.payload())
        return _writable(self._f, "payload_mut")[off + start:off + n]

    def packet_size(self):
        """PacketSize::packet_size: UDP 8, TCP 20 + tcp_options_length (tcp.rs:228-236),
        ICMP / ICMPv6 4 (their payloads have no length function)."""
        if self.kind == "tcp":
            do = self._tcp_data_offset(self.packet())
            return 20 + (do * 4 - 20 if do > 5 else 0)
        return _L4_HEADER[self.kind]

    def get_options_raw(self):
        """TcpPacket::get_options_raw: bytes [20, 20 + options length) of the slice, bounded."""
        if self.kind != "tcp":
            raise AttributeError("options are a TCP field")
        p = self.packet()
        return p[20:min(self.packet_size(), len(p))]

    def get_options_iter(self):
        """TcpPacket::get_options_iter (tcp.rs:68): TcpOption items."""
        return _option_iter(self.get_options_raw(), tcp=True)

    def get_options(self):
        return list(self.get_options_iter())

    def from_packet(self):
        """FromPacket::from_packet: the owned Udp / Tcp / Icmp / Icmpv6 struct as a dict."""
        p = self.packet()
        out = {}
        if self.kind in ("udp", "tcp"):
            out.update(source=self.get_source(), destination=self.get_destination())
        else:
            t = self.get_source()
            out.update({("icmp_type" if self.kind == "icmp" else "icmpv6_type"): t >> 8,
                        ("icmp_code" if self.kind == "icmp" else "icmpv6_code"): t & 0xFF})
        if self.kind == "udp":
            out["length"] = int(self._rec("udp_length")) if _has(self._r, "udp_length") else _be16(p, 4)
        if self.kind == "tcp":
            col = lambda c, fb: int(self._rec(c)) if _has(self._r, c) else fb   # noqa: E731
            do = self._tcp_data_offset(p)
            out.update(sequence=col("tcp_sequence", int.from_bytes(bytes(p[4:8]), "big")),
                       acknowledgement=col("tcp_acknowledgement", int.from_bytes(bytes(p[8:12]), "big")),
                       data_offset=do, reserved=col("tcp_reserved", p[12] & 15), flags=col("tcp_flags", p[13]),
                       window=col("tcp_window", _be16(p, 14)), urgent_ptr=col("tcp_urgent_ptr", _be16(p, 18)),
                       options=self.get_options())
        out["checksum"] = self.get_checksum()
        out["payload"] = bytes(self.payload())
        return out

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

    # ---- the ICMP message views the reference defines over an IcmpPacket's
    # bytes (icmp.rs:153-437; icmpv6.rs:837-995), each None unless the type is
    # its own and the slice holds its 8-B fixed part
    def _icmp_sub(self, cls, types):
        if self.kind not in ("icmp", "icmpv6") or self.get_icmp_type() not in types:
            return None
        return cls(self) if len(self.packet()) >= 8 else None

    def echo_request(self):
        """echo_request::EchoRequestPacket (ICMP type 8, icmp.rs:304-314; ICMPv6 128)."""
        return self._icmp_sub(EchoView, (8,) if self.kind == "icmp" else (128,))

    def echo_reply(self):
        """echo_reply::EchoReplyPacket (ICMP type 0, icmp.rs:221-232; ICMPv6 129)."""
        return self._icmp_sub(EchoView, (0,) if self.kind == "icmp" else (129,))

    def destination_unreachable(self):
        """destination_unreachable::DestinationUnreachablePacket (ICMP type 3, icmp.rs:378-389)."""
        return self._icmp_sub(DestinationUnreachableView, (3,)) if self.kind == "icmp" else None

    def time_exceeded(self):
        """time_exceeded::TimeExceededPacket (ICMP type 11, icmp.rs:425-436)."""
        return self._icmp_sub(TimeExceededView, (11,)) if self.kind == "icmp" else None

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


class _IcmpMessage:
    """Common part of the ICMP message views: type, code, checksum, then 4
    message-specific bytes, payload from byte 8 (packet_size 8)."""

    def __init__(self, icmp):
        self._icmp = icmp

    def minimum_packet_size(self):
        """8: the fixed part of every ICMP message view (icmp.rs:221-232,304-314,378-389,425-436)."""
        return 8

    def to_immutable(self):
        return type(self)(self._icmp.to_immutable())

    consume_to_immutable = to_immutable

    def clone_from(self, other):
        self._icmp.clone_from(other)

    def packet(self):
        return self._icmp.packet()

    def payload(self):
        return self.packet()[8:]

    def packet_mut(self):
        return self._icmp.packet_mut()

    def payload_mut(self):
        return self._icmp.packet_mut()[8:]

    def packet_size(self):
        return 8

    def get_icmp_type(self):
        return self._icmp.get_icmp_type()

    def get_icmp_code(self):
        return self._icmp.get_icmp_code()

    def get_checksum(self):
        return self._icmp.get_checksum()


class EchoView(_IcmpMessage):
    """EchoRequest / EchoReply: identifier (+4), sequence_number (+6), the GPU's columns."""

    def get_identifier(self):
        return self._icmp.get_identifier()

    def get_sequence_number(self):
        return self._icmp.get_sequence_number()

    def from_packet(self):
        return dict(icmp_type=self.get_icmp_type(), icmp_code=self.get_icmp_code(), checksum=self.get_checksum(),
                    identifier=self.get_identifier(), sequence_number=self.get_sequence_number(),
                    payload=bytes(self.payload()))


class DestinationUnreachableView(_IcmpMessage):
    """DestinationUnreachable: unused u16be (+4), next_hop_mtu u16be (+6), payload = the
    quoted IP header + 64 bits of the original datagram."""

    def get_unused(self):
        return _be16(self.packet(), 4)

    def get_next_hop_mtu(self):
        return _be16(self.packet(), 6)

    def from_packet(self):
        return dict(icmp_type=self.get_icmp_type(), icmp_code=self.get_icmp_code(), checksum=self.get_checksum(),
                    unused=self.get_unused(), next_hop_mtu=self.get_next_hop_mtu(), payload=bytes(self.payload()))


class TimeExceededView(_IcmpMessage):
    """TimeExceeded: unused u32be (+4), payload = the quoted datagram."""

    def get_unused(self):
        return int.from_bytes(bytes(self.packet()[4:8]), "big")

    def from_packet(self):
        return dict(icmp_type=self.get_icmp_type(), icmp_code=self.get_icmp_code(), checksum=self.get_checksum(),
                    unused=self.get_unused(), payload=bytes(self.payload()))


class IpView(_PacketTraits):
    """Ipv4Packet / Ipv6Packet over the Ethernet payload."""

    def __init__(self, version, records, i, frame):
        self.version, self._r, self._i, self._f = version, records, i, frame

    def minimum_packet_size(self):
        """Ipv4Packet 20, Ipv6Packet 40."""
        return MINIMUM_PACKET_SIZE["ipv4" if self.version == 4 else "ipv6"]

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

    def _l3(self):
        return int(self._rec("l3_offset")) if _has(self._r, "l3_offset") else 14

    def packet(self):
        """Ipv4Packet / Ipv6Packet::packet(): the buffer the view was built over,
        eth.payload() = the frame from the IP header on."""
        return memoryview(self._f)[self._l3():]

    def packet_mut(self):
        return _writable(self._f, "packet_mut")[self._l3():]

    def payload_mut(self):
        off, n = int(self._rec("l4_offset")), int(self._rec("l4_length"))
        return _writable(self._f, "payload_mut")[off:off + n]

    def _ihl(self):
        return int(self._rec("ip_header_length")) if _has(self._r, "ip_header_length") else self.packet()[0] & 15

    def _total_length(self):
        return int(self._rec("ip_total_length")) if _has(self._r, "ip_total_length") else _be16(self.packet(), 2)

    def packet_size(self):
        """PacketSize::packet_size: IPv4 20 + ipv4_options_length + ipv4_payload_length
        (ipv4.rs:226-243; equals total_length for IHL >= 5, ipv4.rs:316); IPv6
        40 + payload_length (ipv6.rs:34)."""
        if self.version == 4:
            ihl4 = self._ihl() * 4
            return 20 + max(ihl4 - 20, 0) + max(self._total_length() - ihl4, 0)
        pl = int(self._rec("ip6_payload_length")) if _has(self._r, "ip6_payload_length") else _be16(self.packet(), 4)
        return 40 + pl

    def get_options_raw(self):
        """Ipv4Packet::get_options_raw: bytes [20, 20 + options length) of the IP
        packet, bounded by the buffer (decorator.rs:1128-1140)."""
        if self.version != 4:
            raise AttributeError("options are an IPv4 field")
        p = self.packet()
        return p[20:min(20 + max(self._ihl() * 4 - 20, 0), len(p))]

    def get_options_iter(self):
        """Ipv4Packet::get_options_iter (ipv4.rs:156-157): Ipv4Option items."""
        return _option_iter(self.get_options_raw(), tcp=False)

    def get_options(self):
        return list(self.get_options_iter())

    def from_packet(self):
        """FromPacket::from_packet: the owned Ipv4 / Ipv6 struct (every field) as a dict."""
        p = self.packet()
        col = lambda c, fb: int(self._rec(c)) if _has(self._r, c) else fb   # noqa: E731
        if self.version == 4:
            return dict(version=col("ip_version", p[0] >> 4), header_length=self._ihl(),
                        dscp=col("ip_dscp", p[1] >> 2), ecn=col("ip_ecn", p[1] & 3),
                        total_length=self._total_length(), identification=col("ip_identification", _be16(p, 4)),
                        flags=col("ip_flags", p[6] >> 5), fragment_offset=col("ip_fragment_offset", _be16(p, 6) & 0x1FFF),
                        ttl=self.get_ttl(), next_level_protocol=self.get_next_level_protocol(),
                        checksum=_be16(p, 10), source=self.get_source(), destination=self.get_destination(),
                        options=self.get_options(), payload=bytes(self.payload()))
        return dict(version=col("ip_version", p[0] >> 4),
                    traffic_class=col("ip6_traffic_class", ((p[0] & 15) << 4) | (p[1] >> 4)),
                    flow_label=col("ip6_flow_label", ((p[1] & 15) << 16) | _be16(p, 2)),
                    payload_length=col("ip6_payload_length", _be16(p, 4)), next_header=p[6], hop_limit=p[7],
                    source=self.get_source(), destination=self.get_destination(), payload=bytes(self.payload()))

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


class FrameView(_PacketTraits):
    """EthernetPacket over one processed frame."""

    def __init__(self, records, i, frame):
        self._r, self._i, self._f = records, i, frame

    @staticmethod
    def minimum_packet_size():
        """EthernetPacket::minimum_packet_size: 14."""
        return MINIMUM_PACKET_SIZE["ethernet"]

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

    def packet(self):
        """EthernetPacket::packet(): the whole frame."""
        return memoryview(self._f)

    def payload(self):
        """EthernetPacket::payload(): bytes 14.. (the payload has no length function)."""
        return memoryview(self._f)[14:]

    def packet_mut(self):
        return _writable(self._f, "packet_mut")

    def payload_mut(self):
        return _writable(self._f, "payload_mut")[14:]

    def packet_size(self):
        """PacketSize::packet_size: 14 (ethernet.rs:20-30, fixed fields only)."""
        return 14

    def from_packet(self):
        """FromPacket::from_packet: the owned Ethernet struct as a dict."""
        return dict(destination=self.get_destination(), source=self.get_source(),
                    ethertype=_be16(self._f, 12), payload=bytes(self.payload()))

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
