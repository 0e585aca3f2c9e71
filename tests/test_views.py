"""pnet_packet-style views over per-frame records (libpnet_amd.views): the
constructors answer None exactly where the records say the Rust new() failed,
the getters return the record fields and the frame bytes at the recorded
bounds. CPU: over the oracle's records (the views are host logic); GPU: over
a ring batch's records."""
import ipaddress

import numpy as np
import pytest

import libpnet_amd as lp
from libpnet_amd.views import ST
from oracle import coracle, pyoracle
from tests import framegen


def check_views(records, frames, flags=0):
    seen = {"ipv4": 0, "ipv6": 0, "udp": 0, "tcp": 0, "icmp": 0}
    for i, f in enumerate(frames):
        v = lp.frame_view(records, i, f)
        st = int(records["status"][i])
        assert v.valid() == (not st & (ST["ETH_MALFORMED"] | ST["DESC_INVALID"]))
        ip4, ip6 = v.ipv4(), v.ipv6()
        assert (ip4 is not None) == ((st & 3) == 1 and not st & ST["L3_MALFORMED"])
        assert (ip6 is not None) == ((st & 3) == 2 and not st & ST["L3_MALFORMED"])
        ip = ip4 or ip6
        if ip is None:
            continue
        seen["ipv4" if ip4 else "ipv6"] += 1
        l3 = int(records["l3_offset"][i])
        if "ip_version" in (getattr(records, "dtype", None) and records.dtype.names or records):
            hdr = pyoracle.getters(f[l3:], pyoracle.IPV4 if ip4 else pyoracle.IPV6)
            assert ip.get_version() == hdr["ip_version"]
            if ip4:
                assert (ip.get_header_length(), ip.get_dscp(), ip.get_ecn(), ip.get_total_length(),
                        ip.get_identification(), ip.get_flags(), ip.get_fragment_offset()) == tuple(
                    hdr[k] for k in ("ip_header_length", "ip_dscp", "ip_ecn", "ip_total_length",
                                     "ip_identification", "ip_flags", "ip_fragment_offset"))
            else:
                assert (ip.get_traffic_class(), ip.get_flow_label(), ip.get_payload_length()) == (
                    hdr["ip6_traffic_class"], hdr["ip6_flow_label"], hdr["ip6_payload_length"])
            assert v.get_destination() == bytes(f[0:6]) and v.get_source() == bytes(f[6:12])
        if ip4:
            assert ip.get_source() == ipaddress.IPv4Address(bytes(f[l3 + 12:l3 + 16]))
            assert ip.get_destination() == ipaddress.IPv4Address(bytes(f[l3 + 16:l3 + 20]))
            assert ip.checksum_ok() == bool(st & ST["IP_CSUM_OK"])
        else:
            assert ip.get_source() == ipaddress.IPv6Address(bytes(f[l3 + 8:l3 + 24]))
        off, n = int(records["l4_offset"][i]), int(records["l4_length"][i])
        assert bytes(ip.payload()) == bytes(f[off:off + n])
        for kind in ("udp", "tcp", "icmp"):
            l4 = getattr(ip, kind)()
            if l4 is None:
                continue
            seen[kind] += 1
            p = bytes(l4.packet())
            if kind in ("udp", "tcp"):
                assert l4.get_source() == (p[0] << 8 | p[1]) and l4.get_destination() == (p[2] << 8 | p[3])
            if "tcp_sequence" in (getattr(records, "dtype", None) and records.dtype.names or records):
                if kind == "udp":
                    assert l4.get_length() == (p[4] << 8 | p[5])
                elif kind == "tcp":
                    t = pyoracle.getters(p, pyoracle.TCP)
                    assert (l4.get_sequence(), l4.get_acknowledgement(), l4.get_data_offset(), l4.get_reserved(),
                            l4.get_flags(), l4.get_window(), l4.get_urgent_ptr()) == tuple(
                        t[k] for k in ("tcp_sequence", "tcp_acknowledgement", "tcp_data_offset", "tcp_reserved",
                                       "tcp_flags", "tcp_window", "tcp_urgent_ptr"))
                elif len(p) >= 8:
                    assert l4.get_identifier() == (p[4] << 8 | p[5]) and l4.get_sequence_number() == (p[6] << 8 | p[7])
            else:
                assert l4.get_icmp_type() == p[0] and l4.get_icmp_code() == p[1]
            assert l4.checksum_ok() == bool(st & ST["L4_CSUM_OK"])
            c = l4.computed_checksum()
            assert c is None or c == int(records["l4_csum"][i])
            assert bytes(l4.payload()) == p[{"udp": 8, "icmp": 4}.get(kind, len(p) - len(bytes(l4.payload()))):]
    return seen


def test_views_over_oracle_records():
    rng = np.random.default_rng(14)
    frames = framegen.edge_frames(rng) + framegen.random_frames(rng, 3000)
    buf, offs, lens = framegen.pack(frames)
    rec = coracle.rx_batch(buf, len(frames), offsets=offs, lengths=lens)
    seen = check_views(rec, frames)
    assert min(seen.values()) > 50, seen


def test_tcp_payload_skips_options():
    rng = np.random.default_rng(15)
    f = bytearray(framegen.build_frame(rng, "tcp", 60))
    f[14 + 20 + 12] = (8 << 4)                    # data offset 8: 12 B of options
    rec = coracle.rx_batch(np.frombuffer(bytes(f) + bytes(32), np.uint8), 1, offsets=np.array([0], np.uint64),
                           lengths=np.array([len(f)], np.uint32))
    tcp = lp.frame_view(rec, 0, bytes(f)).ipv4().tcp()
    assert bytes(tcp.payload()) == bytes(f[14 + 20 + 32:])


def test_missing_column_is_an_error():
    rng = np.random.default_rng(16)
    f = framegen.build_frame(rng, "udp", 20)
    rec = {"status": np.array([pyoracle.rx_frame(f)["status"]], np.uint16)}
    with pytest.raises(KeyError):
        lp.frame_view(rec, 0, f).ipv4().get_source()


@pytest.mark.gpu
def test_views_over_ring_batch(tmp_path):
    rng = np.random.default_rng(17)
    frames = framegen.random_frames(rng, 4000)
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=1000, columns=lp.ALL_COLUMNS)
    batches = []
    for f in frames:
        batches.extend(ring.feed(f))
    batches.extend(ring.drain())
    batches.sort(key=lambda b: b.id)
    i0 = 0
    for b in batches:
        fr = [b.frames[int(b.offsets[k]):int(b.offsets[k]) + int(b.lengths[k])] for k in range(b.n)]
        assert [bytes(x) for x in fr] == frames[i0:i0 + b.n]
        check_views(b.records, fr)
        i0 += b.n
    assert i0 == len(frames)
