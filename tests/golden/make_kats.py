#!/usr/bin/env python3
"""Writes tests/golden/reference_kats.json — the reference's known-answer vectors.

Every vector below re-builds, byte for byte, the input that one of libpnet's
own unit tests constructs (by following that test's setter calls), and records
the value that test asserts. Nothing from the reference is imported or run
(it is Rust, and no Rust toolchain exists here); the expected values are the
literal constants in the cited assertions. Vectors marked "derived" have no
reference assertion: their expected values come from this repo's oracle and
are pinned only transitively ("Derived").

Run:  python tests/golden/make_kats.py   (rewrites the JSON next to this file)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def hx(b):
    return bytes(b).hex()


def kat(name, kind, source, expected, **kw):
    d = {"name": name, "kind": kind, "source": source, "expected": expected}
    for k, v in kw.items():
        d[k] = hx(v) if isinstance(v, (bytes, bytearray)) else v
    return d


def main():
    v = []
    # ---- util.rs:189-198 sum_be_words_different_skipwords -----------------
    data = bytes(range(11))
    for skip, exp in ((1, 7190), (2, 6676), (99, 7705), (101, 7705)):
        v.append(kat(f"sum_be_words_0..11_skip{skip}", "sum_be_words",
                     "pnet_packet/src/util.rs:190-198", exp, data=data, skipword=skip))
    # ---- util.rs:218-237 misaligned ptr: a 12-byte slice at an odd address,
    # bytes 0..10 = i, byte 11 = 0 (from vec![0; 13]) --------------------------
    data12 = bytes(range(11)) + b"\x00"
    for skip, exp in ((1, 7190), (2, 6676), (99, 7705), (101, 7705)):
        v.append(kat(f"sum_be_words_misaligned_skip{skip}", "sum_be_words",
                     "pnet_packet/src/util.rs:218-237", exp, data=data12, skipword=skip,
                     misalign=1))
    # ---- util.rs:200-216 sum_be_words_small_sizes ---------------------------
    for d, skip, exp in ((b"", 0, 0), (b"", 10, 0), (b"\x01", 1, 256), (b"\x01\x01", 0, 0),
                         (b"\x01\x01", 1, 257), (b"\x04" * 3, 0, 1024), (b"\x04" * 3, 1, 1028),
                         (b"\x04" * 3, 2, 2052), (b"\x04" * 3, 3, 2052)):
        v.append(kat(f"sum_be_words_len{len(d)}_skip{skip}", "sum_be_words",
                     "pnet_packet/src/util.rs:200-216", exp, data=d, skipword=skip))

    # ---- ipv4.rs:185-223 ipv4::checksum ------------------------------------
    # set_header_length(x) writes the low nibble of byte 0 (u4 at bit offset 4).
    def with_ihl(buf, ihl):
        b = bytearray(buf)
        b[0] = (b[0] & 0xF0) | (ihl & 0x0F)
        return b

    def with_csum(buf, c):
        b = bytearray(buf)
        b[10], b[11] = c >> 8, c & 0xFF
        return b

    z = with_ihl(bytes(20), 5)
    v.append(kat("ipv4_checksum_zeros", "ipv4_header", "pnet_packet/src/ipv4.rs:186-191",
                 64255, data=z))
    v.append(kat("ipv4_checksum_zeros_set123", "ipv4_header", "pnet_packet/src/ipv4.rs:192-193",
                 64255, data=with_csum(z, 123)))
    f = with_ihl(b"\xff" * 20, 5)
    v.append(kat("ipv4_checksum_nonzero", "ipv4_header", "pnet_packet/src/ipv4.rs:197-202",
                 2560, data=f))
    v.append(kat("ipv4_checksum_nonzero_set123", "ipv4_header", "pnet_packet/src/ipv4.rs:203-204",
                 2560, data=with_csum(f, 123)))
    v.append(kat("ipv4_checksum_too_small_ihl", "ipv4_header", "pnet_packet/src/ipv4.rs:208-214",
                 51910, data=with_ihl(bytes([148] * 20), 0)))
    v.append(kat("ipv4_checksum_too_large_ihl", "ipv4_header", "pnet_packet/src/ipv4.rs:217-223",
                 51142, data=with_ihl(bytes([148] * 20), 99)))
    # ipv4.rs:292-357 ipv4_packet_test: 200-byte buffer, ref_packet header
    hdr = bytes([0x45, 0x11, 0x00, 0x73, 0x01, 0x01, 0x41, 0x01, 0x40, 0x11, 0x00, 0x00,
                 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7])
    v.append(kat("ipv4_packet_test", "ipv4_header", "pnet_packet/src/ipv4.rs:340-356",
                 0xB64E, data=hdr + bytes(180)))

    # ---- ipv4 payload bounds (decorator.rs:728-753 + ipv4.rs:241-243) -------
    p = bytearray(30)
    p[0] = 0x05
    p[2:4] = (20).to_bytes(2, "big")
    v.append(kat("ipv4_payload_length_20", "ipv4_payload_len", "pnet_packet/src/ipv4.rs:245-251",
                 0, data=p))
    p[2:4] = (30).to_bytes(2, "big")
    v.append(kat("ipv4_payload_length_30", "ipv4_payload_len", "pnet_packet/src/ipv4.rs:254-255",
                 10, data=p))
    q = bytearray(hdr + bytes(180))
    v.append(kat("ipv4_packet_test_payload_len", "ipv4_payload_len",
                 "pnet_packet/src/ipv4.rs:313-315", 95, data=q))

    # ---- udp.rs:58-100 udp_header_ipv4_test --------------------------------
    udp = bytes([0x30, 0x39, 0xd4, 0x31, 0x00, 0x0c, 0x00, 0x00]) + b"test"
    v.append(kat("udp_ipv4_checksum", "ipv4_checksum", "pnet_packet/src/udp.rs:58-100",
                 0x9178, data=udp, skipword=3, src=[192, 168, 0, 1], dst=[192, 168, 0, 199],
                 proto=17))
    # ---- udp.rs:128-170 udp_header_ipv6_test --------------------------------
    lo6 = [0] * 15 + [1]
    v.append(kat("udp_ipv6_checksum", "ipv6_checksum", "pnet_packet/src/udp.rs:128-170",
                 0x1390, data=udp, skipword=3, src=lo6, dst=lo6, proto=17))
    # ---- tcp.rs:288-357 tcp_header_ipv4_test (checksum field zero before compute)
    tcp = bytes([0xc1, 0x67, 0x23, 0x28, 0x90, 0x37, 0xd2, 0xb8, 0x94, 0x4b, 0xb2, 0x76,
                 0x80, 0x18, 0x0f, 0xaf, 0x00, 0x00, 0x00, 0x00, 0x01, 0x01, 0x08, 0x0a,
                 0x2c, 0x57, 0xcd, 0xa5, 0x02, 0xa0, 0x41, 0x92]) + b"test"
    v.append(kat("tcp_ipv4_checksum", "ipv4_checksum", "pnet_packet/src/tcp.rs:288-357",
                 0xC031, data=tcp, skipword=8, src=[192, 168, 2, 1], dst=[192, 168, 111, 51],
                 proto=6))
    # ---- icmp.rs:82-108 ----------------------------------------------------
    v.append(kat("icmp_checksum_zeros", "checksum", "pnet_packet/src/icmp.rs:82-89",
                 65535, data=bytes(8), skipword=1))
    v.append(kat("icmp_checksum_zeros_set123", "checksum", "pnet_packet/src/icmp.rs:88-89",
                 65535, data=bytes([0, 0, 0, 123, 0, 0, 0, 0]), skipword=1))
    v.append(kat("icmp_checksum_nonzero", "checksum", "pnet_packet/src/icmp.rs:92-99",
                 0, data=b"\xff" * 8, skipword=1))
    v.append(kat("icmp_checksum_nonzero_set0", "checksum", "pnet_packet/src/icmp.rs:97-98",
                 0, data=b"\xff\xff\x00\x00" + b"\xff" * 4, skipword=1))
    v.append(kat("icmp_checksum_odd", "checksum", "pnet_packet/src/icmp.rs:101-107",
                 49535, data=bytes([191] * 7), skipword=1))
    # ---- icmpv6.rs:88-117 ---------------------------------------------------
    echo = bytes([0x80, 0x00, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01,
                  0x20, 0x20, 0x75, 0x73, 0x74, 0x20, 0x61, 0x20,
                  0x66, 0x6c, 0x65, 0x73, 0x68, 0x20, 0x77, 0x6f,
                  0x75, 0x6e, 0x64, 0x20, 0x20, 0x74, 0x69, 0x73,
                  0x20, 0x62, 0x75, 0x74, 0x20, 0x61, 0x20, 0x73,
                  0x63, 0x72, 0x61, 0x74, 0x63, 0x68, 0x20, 0x20,
                  0x6b, 0x6e, 0x69, 0x67, 0x68, 0x74, 0x73, 0x20,
                  0x6f, 0x66, 0x20, 0x6e, 0x69, 0x20, 0x20, 0x20])
    v.append(kat("icmpv6_echo_request", "ipv6_checksum", "pnet_packet/src/icmpv6.rs:88-110",
                 0x1D2E, data=echo, skipword=1, src=lo6, dst=lo6, proto=58))
    v.append(kat("icmpv6_echo_reply_type", "ipv6_checksum", "pnet_packet/src/icmpv6.rs:112-115",
                 0x1C2E, data=bytes([0x81]) + echo[1:], skipword=1, src=lo6, dst=lo6, proto=58))

    # ---- ethernet.rs:32-54 field layout -------------------------------------
    eth = bytes([0xde, 0xf0, 0x12, 0x34, 0x45, 0x67, 0x12, 0x34, 0x56, 0x78, 0x9a, 0xbc,
                 0x86, 0xdd])
    v.append(kat("ethernet_header_test", "ethernet_fields", "pnet_packet/src/ethernet.rs:32-54",
                 {"destination": "def012344567", "source": "123456789abc", "ethertype": 0x86DD},
                 data=eth))
    # ---- ipv6.rs:147+ payload bounded by payload_length ----------------------
    ip6 = bytearray(0x200)
    ip6[0] = 0x61
    ip6[4:6] = (0x0101).to_bytes(2, "big")
    v.append(kat("ipv6_header_payload_len", "ipv6_payload_len", "pnet_packet/src/ipv6.rs:164-166",
                 0x0101, data=ip6))
    # ---- tcp.rs:421-433 payload with invalid data offset --------------------
    t20 = bytearray(20)
    t20[12] = 10 << 4
    v.append(kat("tcp_payload_invalid_offset", "tcp_payload_len", "pnet_packet/src/tcp.rs:421-433",
                 0, data=t20))

    # ---- header-field getters: the values the reference's tests assert after
    # their setter calls, over the bytes the same tests assert were written ----
    v.append(kat("ethernet_getters", "getters", "pnet_packet/src/ethernet.rs:33-54",
                 {"eth_dst": 0xDEF012344567, "eth_src": 0x123456789ABC}, view="ethernet", data=eth))
    v.append(kat("ipv4_getters", "getters", "pnet_packet/src/ipv4.rs:292-357",
                 {"ip_version": 4, "ip_header_length": 5, "ip_dscp": 4, "ip_ecn": 1, "ip_total_length": 115,
                  "ip_identification": 257, "ip_flags": 2, "ip_fragment_offset": 257, "ttl": 64, "ip_proto": 17},
                 view="ipv4", data=hdr))
    ip6h = bytes([0x61, 0x11, 0x01, 0x01, 0x01, 0x01, 0x00, 0x01]) + bytes([0x01, 0x10, 0x10, 0x01] * 8)
    v.append(kat("ipv6_getters", "getters", "pnet_packet/src/ipv6.rs:147-180,270-290",
                 {"ip_version": 6, "ip6_traffic_class": 17, "ip6_flow_label": 0x10101,
                  "ip6_payload_length": 0x0101, "ttl": 1, "ip_proto": 0}, view="ipv6", data=ip6h))
    v.append(kat("udp_getters", "getters", "pnet_packet/src/udp.rs:59-100",
                 {"src_port": 12345, "dst_port": 54321, "udp_length": 12}, view="udp", data=udp))
    v.append(kat("tcp_getters", "getters", "pnet_packet/src/tcp.rs:288-357",
                 {"src_port": 49511, "dst_port": 9000, "tcp_sequence": 0x9037D2B8,
                  "tcp_acknowledgement": 0x944BB276, "tcp_data_offset": 8, "tcp_reserved": 0,
                  "tcp_flags": 0x18, "tcp_window": 4015, "tcp_urgent_ptr": 0},
                 view="tcp", data=tcp))
    # echo identifier / sequence_number over the icmpv6.rs:88-110 echo request
    # bytes: layout-derived (icmp.rs:221-232,303-314), no reference assertion
    v.append(kat("icmpv6_echo_getters", "getters", "pnet_packet/src/icmp.rs:303-314 layout (derived)",
                 {"src_port": 0x8000, "dst_port": 0, "icmp_sequence": 1}, view="icmpv6", data=echo,
                 derived=True))

    # ---- derived (no reference assertion) -------------
    # benches/rs_sender.rs:25-101: the 64-B Eth/IPv4/UDP frame, dst/src MAC zero
    fr = bytearray(64)
    fr[12:14] = b"\x08\x00"
    ip = fr[14:]
    ip[0] = 0x45
    ip[2:4] = (33).to_bytes(2, "big")
    ip[8] = 4
    ip[9] = 17
    ip[12:16] = bytes([127, 0, 0, 1])
    ip[16:20] = bytes([127, 0, 0, 1])
    ip[20:22] = (1234).to_bytes(2, "big")
    ip[22:24] = (1234).to_bytes(2, "big")
    ip[24:26] = (13).to_bytes(2, "big")
    ip[28:33] = b"rmesg"
    ip[10:12] = (0xB8CA).to_bytes(2, "big")
    ip[26:28] = (0xB94C).to_bytes(2, "big")
    fr[14:] = ip
    v.append(kat("rs_sender_frame", "rx_frame", "benches/rs_sender.rs:25-101 (derived)",
                 {"ip_csum": 0xB8CA, "l4_csum": 0xB94C, "ip_ok": True, "l4_ok": True,
                  "l4_offset": 34, "l4_length": 13, "src_port": 1234, "dst_port": 1234},
                 data=fr, derived=True))
    # pnet_packet/benches/packet_benchmarks.rs:63 captured TCP frame (TX-offload partial)
    cap = bytes.fromhex("000c291ce319ecf4bbd93e7d08004500002e1b6540008006cd76c0a8c887c0a8c815"
                        "1a3707d0dd6abb2b1f5fd25150180402120f000068656c6c6f0a")
    v.append(kat("captured_tcp_frame", "rx_frame",
                 "pnet_packet/benches/packet_benchmarks.rs:63 (derived)",
                 {"ip_csum": 0xCD76, "l4_csum": 0xA9AB, "ip_ok": True, "l4_ok": False,
                  "l4_offset": 34, "l4_length": 26, "src_port": 0x1A37, "dst_port": 0x07D0},
                 data=cap, derived=True))

    with open(os.path.join(HERE, "reference_kats.json"), "w") as fh:
        json.dump({"generator": "tests/golden/make_kats.py", "vectors": v}, fh, indent=1)
    print(f"wrote {len(v)} vectors")


if __name__ == "__main__":
    main()
