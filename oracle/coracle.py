"""ctypes binding to the C parity oracle (oracle/libpnet_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the libpnet_amd product package.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpnet_oracle.so")

REC_DTYPE = np.dtype([
    ("status", "<u2"), ("ip_csum", "<u2"), ("l4_csum", "<u2"), ("ethertype", "<u2"),
    ("ip_proto", "u1"), ("ttl", "u1"), ("l4_offset", "<u2"), ("l4_length", "<u2"),
    ("src_port", "<u2"), ("dst_port", "<u2"), ("_pad", "<u2"),
    ("src_ipv4", "<u4"), ("dst_ipv4", "<u4"),
    ("src_ipv6", "u1", (16,)), ("dst_ipv6", "u1", (16,)),
    ("vlan_tci", "<u2"), ("l3_offset", "u1"), ("_pad2", "u1"),
    ("eth_dst", "<u8"), ("eth_src", "<u8"),
    ("tcp_sequence", "<u4"), ("tcp_acknowledgement", "<u4"), ("ip6_flow_label", "<u4"),
    ("ip_total_length", "<u2"), ("ip_identification", "<u2"), ("ip_fragment_offset", "<u2"),
    ("ip6_payload_length", "<u2"), ("udp_length", "<u2"), ("tcp_window", "<u2"), ("tcp_urgent_ptr", "<u2"),
    ("icmp_sequence", "<u2"),
    ("ip_version", "u1"), ("ip_header_length", "u1"), ("ip_dscp", "u1"), ("ip_ecn", "u1"), ("ip_flags", "u1"),
    ("ip6_traffic_class", "u1"), ("tcp_data_offset", "u1"), ("tcp_reserved", "u1"), ("tcp_flags", "u1"),
    ("_pad3", "u1", (3,)),
], align=True)

RX_VLAN, RX_IPV6_EXT, RX_L3 = 0x1, 0x2, 0x4

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_sum_be_words.restype = ctypes.c_uint32
        L.oracle_sum_be_words.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t]
        L.oracle_checksum.restype = ctypes.c_uint16
        L.oracle_checksum.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t]
        for f in (L.oracle_ipv4_checksum, L.oracle_ipv6_checksum):
            f.restype = ctypes.c_uint16
            f.argtypes = [u8p, ctypes.c_size_t, ctypes.c_size_t, u8p, ctypes.c_size_t,
                          u8p, u8p, ctypes.c_uint8]
        L.oracle_rx_frame.restype = None
        L.oracle_rx_frame.argtypes = [u8p, ctypes.c_size_t, ctypes.c_void_p]
        L.oracle_rx_frame_ex.restype = None
        L.oracle_rx_frame_ex.argtypes = [u8p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_rx_batch_ex.restype = None
        L.oracle_rx_batch_ex.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_int]
        L.oracle_rx_batch.restype = None
        L.oracle_rx_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int]
        L.oracle_tx_fill.restype = None
        L.oracle_tx_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint32, ctypes.c_void_p]
        L.oracle_rx_batch_reps.restype = None
        L.oracle_rx_batch_reps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.oracle_rs_sender_build.restype = None
        L.oracle_rs_sender_build.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.oracle_checksum_slices_reps.restype = None
        L.oracle_checksum_slices_reps.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.oracle_checksum_slices.restype = None
        L.oracle_checksum_slices.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib = L
    return _lib


def _buf(b):
    b = bytes(b)
    arr = (ctypes.c_uint8 * max(1, len(b))).from_buffer_copy(b if b else b"\0")
    return arr


def sum_be_words(data, skipword):
    return lib().oracle_sum_be_words(_buf(data), len(data), skipword)


def checksum(data, skipword):
    return lib().oracle_checksum(_buf(data), len(data), skipword)


def ipv4_checksum(data, skipword, extra, src, dst, proto):
    return lib().oracle_ipv4_checksum(_buf(data), len(data), skipword, _buf(extra), len(extra),
                                      _buf(src), _buf(dst), proto)


def ipv6_checksum(data, skipword, extra, src, dst, proto):
    return lib().oracle_ipv6_checksum(_buf(data), len(data), skipword, _buf(extra), len(extra),
                                      _buf(src), _buf(dst), proto)


def rx_frame(frame, flags=0):
    rec = np.zeros(1, dtype=REC_DTYPE)
    lib().oracle_rx_frame_ex(_buf(frame), len(frame), flags, rec.ctypes.data)
    return rec[0]


def rx_batch(buf, n, *, stride=0, frame_len=0, first=0, offsets=None, lengths=None,
             nthreads=1, flags=0):
    """Oracle records for a frame batch held in a numpy uint8 array."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    out = np.zeros(n, dtype=REC_DTYPE)
    offp = lenp = None
    if stride == 0:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        offp, lenp = offsets.ctypes.data, lengths.ctypes.data
    lib().oracle_rx_batch_ex(buf.ctypes.data, buf.size, n, first, stride, frame_len,
                             offp, lenp, flags, out.ctypes.data, nthreads)
    return out


def checksum_slices_reps(buf, offsets, lengths, skipwords, out, nthreads=1, reps=1):
    """util::checksum per slice, persistent threads, each shard `reps` times (CPU baseline timing)."""
    lib().oracle_checksum_slices_reps(buf.ctypes.data, len(offsets), offsets.ctypes.data, lengths.ctypes.data,
                                      skipwords.ctypes.data, out.ctypes.data, nthreads, reps)
    return out


def checksum_slices(buf, offsets, lengths, skipwords):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    skipwords = np.ascontiguousarray(skipwords, dtype=np.uint32)
    out = np.zeros(len(offsets), dtype=np.uint16)
    lib().oracle_checksum_slices(buf.ctypes.data, len(offsets), offsets.ctypes.data,
                                 lengths.ctypes.data, skipwords.ctypes.data, out.ctypes.data)
    return out


def tx_fill(buf, n, *, stride=0, frame_len=0, first=0, offsets=None, lengths=None, flags=0):
    """Patch a COPY of buf the way the sender side does; returns (patched, records)."""
    out_buf = np.array(buf, dtype=np.uint8, copy=True)
    recs = np.zeros(n, dtype=REC_DTYPE)
    offp = lenp = None
    if stride == 0:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        offp, lenp = offsets.ctypes.data, lengths.ctypes.data
    lib().oracle_tx_fill(out_buf.ctypes.data, out_buf.size, n, first, stride, frame_len, offp, lenp,
                         flags, recs.ctypes.data)
    return out_buf, recs


def rx_batch_reps(buf, n, *, stride=0, frame_len=0, first=0, offsets=None, lengths=None, nthreads=1, reps=1,
                  flags=0, out=None):
    """rx_batch with persistent threads, each shard processed `reps` times (CPU baseline timing)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    if out is None:
        out = np.zeros(n, dtype=REC_DTYPE)
    offp = lenp = None
    if stride == 0:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        offp, lenp = offsets.ctypes.data, lengths.ctypes.data
    lib().oracle_rx_batch_reps(buf.ctypes.data, buf.size, n, first, stride, frame_len, offp, lenp, flags,
                               out.ctypes.data, nthreads, reps)
    return out


def rs_sender_build(n, nthreads=1, reps=1, buf=None):
    """n frames built as benches/rs_sender.rs:25-72 does (64-B stride); returns the uint8 buffer."""
    if buf is None:
        buf = np.zeros(64 * n + 32, dtype=np.uint8)
    lib().oracle_rs_sender_build(buf.ctypes.data, n, nthreads, reps)
    return buf
