"""pnet_packet's checksum functions under their reference names, computed on the GPU.

Drop-in shape of the free functions a libpnet user calls per packet, so code
(and tests) written against the reference read the same:

    from libpnet_amd.packet import util, ipv4, udp, tcp, icmp, icmpv6
    util.checksum(data, skipword)                                   # util.rs:76-82
    util.ipv4_checksum(data, skipword, extra_data, src, dst, proto) # util.rs:92-117
    util.ipv6_checksum(data, skipword, extra_data, src, dst, proto) # util.rs:125-150
    ipv4.checksum(ipv4_packet)                                      # ipv4.rs:165-178
    udp.ipv4_checksum(udp_packet, src, dst)  / ipv6_checksum / *_adv(.., extra, ..)  # udp.rs:34-56,104-126
    tcp.ipv4_checksum(tcp_packet, src, dst)  / ipv6_checksum / *_adv                 # tcp.rs:239-286
    icmp.checksum(icmp_packet)                                      # icmp.rs:70-75
    icmpv6.checksum(icmpv6_packet, src, dst)                        # icmpv6.rs:80-85

A packet argument is the bytes of that layer (the reference's `packet.packet()`
slice); addresses are `ipaddress` objects, strings or raw bytes. Every call is
one launch of the batched slice kernels through the C-ABI on the current
device (`set_device`), so these are for API parity and small workloads; batch
work belongs on `rx_process` / the `*_slices` entry points. The `*_many`
variants take lists and make one launch for all of them. There is no CPU
compute path: without a GPU these raise.
"""
import ipaddress

import numpy as np
import torch

from . import engine

_DEVICE = [0]


def set_device(index):
    """GPU used by these functions (default 0)."""
    _DEVICE[0] = int(index)


def _dev():
    return torch.device("cuda", _DEVICE[0])


def _addr(a, n):
    if isinstance(a, (ipaddress.IPv4Address, ipaddress.IPv6Address)):
        b = a.packed
    elif isinstance(a, str):
        b = ipaddress.ip_address(a).packed
    else:
        b = bytes(a)
    if len(b) != n:
        raise ValueError(f"expected a {n}-byte address, got {len(b)} bytes")
    return b


def _pack(datas, extras=None):
    """Concatenate slices (and extra slices) into one device buffer; offsets/lengths."""
    parts, offs, lens, eoffs, elens, pos = [], [], [], [], [], 0
    for d in datas:
        d = bytes(d)
        offs.append(pos)
        lens.append(len(d))
        parts.append(d)
        pos += len(d)
    for e in extras or ():
        e = bytes(e)
        eoffs.append(pos)
        elens.append(len(e))
        parts.append(e)
        pos += len(e)
    host = np.frombuffer(b"".join(parts) + bytes(16), dtype=np.uint8)   # readable to the next 16 B
    dev = _dev()
    buf = torch.from_numpy(host.copy()).to(dev)

    def t(v, dt):
        return torch.tensor(v, dtype=dt, device=dev)
    return buf, t(offs, torch.int64), t(lens, torch.int32), t(eoffs, torch.int64), t(elens, torch.int32)


def _u16(t):
    torch.cuda.synchronize(t.device)
    return t.cpu().numpy().view(np.uint16)


class util:
    """pnet_packet::util (re-exported as pnet::util)."""

    @staticmethod
    def checksum_many(datas, skipwords):
        datas = list(datas)
        if not datas:
            return np.zeros(0, np.uint16)
        buf, o, l, _, _ = _pack(datas)
        s = torch.tensor([int(k) for k in skipwords], dtype=torch.int32, device=buf.device)
        return _u16(engine.checksum_slices(buf, o, l, s))

    @staticmethod
    def checksum(data, skipword):
        return int(util.checksum_many([data], [skipword])[0])

    @staticmethod
    def _pseudo_many(version, datas, skipwords, extras, sources, destinations, protos):
        alen = 4 if version == 4 else 16
        datas = list(datas)
        if not datas:
            return np.zeros(0, np.uint16)
        extras = [bytes(e) for e in extras] if extras is not None else [b""] * len(datas)
        addrs = np.frombuffer(b"".join(_addr(s, alen) + _addr(d, alen) for s, d in zip(sources, destinations)),
                              dtype=np.uint8).reshape(len(datas), 2 * alen)
        pr = np.array([int(p) for p in protos], dtype=np.uint8)
        sk = [int(k) for k in skipwords]
        if any(extras):
            buf, o, l, eo, el = _pack(datas, extras)
            dev = buf.device
            out = engine.checksum_adv_slices(version, buf, o, l, torch.tensor(sk, dtype=torch.int32, device=dev),
                                             eo, el, torch.from_numpy(addrs.copy()).to(dev),
                                             torch.from_numpy(pr).to(dev))
        else:
            buf, o, l, _, _ = _pack(datas)
            dev = buf.device
            fn = engine.ipv4_checksum_slices if version == 4 else engine.ipv6_checksum_slices
            out = fn(buf, o, l, torch.tensor(sk, dtype=torch.int32, device=dev),
                     torch.from_numpy(addrs.copy()).to(dev), torch.from_numpy(pr).to(dev))
        return _u16(out)

    @staticmethod
    def ipv4_checksum_many(datas, skipwords, extras, sources, destinations, protos):
        return util._pseudo_many(4, datas, skipwords, extras, sources, destinations, protos)

    @staticmethod
    def ipv6_checksum_many(datas, skipwords, extras, sources, destinations, protos):
        return util._pseudo_many(6, datas, skipwords, extras, sources, destinations, protos)

    @staticmethod
    def ipv4_checksum(data, skipword, extra_data, source, destination, next_level_protocol):
        return int(util.ipv4_checksum_many([data], [skipword], [extra_data], [source], [destination],
                                           [next_level_protocol])[0])

    @staticmethod
    def ipv6_checksum(data, skipword, extra_data, source, destination, next_level_protocol):
        return int(util.ipv6_checksum_many([data], [skipword], [extra_data], [source], [destination],
                                           [next_level_protocol])[0])


class ipv4:
    """pnet_packet::ipv4."""

    @staticmethod
    def checksum(packet):
        """ipv4::checksum: the header length is IHL*4 clamped to [20, len(packet)]
        (ipv4.rs:165-178), the checksum word (index 5) skipped."""
        p = bytes(packet)
        if len(p) < 20:
            raise ValueError("Ipv4Packet::new needs at least 20 bytes")
        hl = min(max((p[0] & 0x0F) * 4, 20), len(p))
        return util.checksum(p[:hl], 5)


def _l4(skip, proto):
    class _L4:
        @staticmethod
        def ipv4_checksum(packet, source, destination):
            return util.ipv4_checksum(packet, skip, b"", source, destination, proto)

        @staticmethod
        def ipv4_checksum_adv(packet, extra_data, source, destination):
            return util.ipv4_checksum(packet, skip, extra_data, source, destination, proto)

        @staticmethod
        def ipv6_checksum(packet, source, destination):
            return util.ipv6_checksum(packet, skip, b"", source, destination, proto)

        @staticmethod
        def ipv6_checksum_adv(packet, extra_data, source, destination):
            return util.ipv6_checksum(packet, skip, extra_data, source, destination, proto)
    return _L4


udp = _l4(3, 17)      # pnet_packet::udp: checksum word 3 (bytes 6..7), IpNextHeaderProtocols::Udp
udp.__doc__ = "pnet_packet::udp (udp.rs:34-56,104-126)."
tcp = _l4(8, 6)       # pnet_packet::tcp: checksum word 8 (bytes 16..17), IpNextHeaderProtocols::Tcp
tcp.__doc__ = "pnet_packet::tcp (tcp.rs:239-286)."


class icmp:
    """pnet_packet::icmp."""

    @staticmethod
    def checksum(packet):
        """icmp::checksum: util::checksum(packet, 1) (icmp.rs:70-75)."""
        return util.checksum(packet, 1)


class icmpv6:
    """pnet_packet::icmpv6."""

    @staticmethod
    def checksum(packet, source, destination):
        """icmpv6::checksum: util::ipv6_checksum(packet, 1, &[], src, dst, Icmpv6) (icmpv6.rs:80-85)."""
        return util.ipv6_checksum(packet, 1, b"", source, destination, 58)


def _host_setup():
    import ctypes
    from ._lib import lib
    vp, u64, u8 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint8
    lib.pnetgpu_util_checksum.restype = ctypes.c_int
    lib.pnetgpu_util_checksum.argtypes = [vp, vp, u64, u64, ctypes.POINTER(ctypes.c_uint16)]
    for fn in (lib.pnetgpu_util_ipv4_checksum, lib.pnetgpu_util_ipv6_checksum):
        fn.restype = ctypes.c_int
        fn.argtypes = [vp, vp, u64, u64, vp, u64, vp, vp, u8, ctypes.POINTER(ctypes.c_uint16)]
    lib.pnetgpu_checksum_slices_host.restype = ctypes.c_int
    lib.pnetgpu_checksum_slices_host.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp]
    return ctypes, lib


class util_host:
    """pnet_packet::util's three functions through the host-memory C-ABI
    (include/pnetgpu_util.h: the entry points a Rust or C caller replacing one
    `util::checksum(&[u8], usize)` call binds): host bytes in, the word out, one
    synchronous staged launch on the context's own stream."""

    @staticmethod
    def _buf(b):
        b = bytes(b)
        return b, (len(b) and b) or None

    @staticmethod
    def checksum(data, skipword):
        ctypes, lib = _host_setup()
        from ._lib import check
        data, p = util_host._buf(data)
        out = ctypes.c_uint16()
        check(lib.pnetgpu_util_checksum(engine.context(_DEVICE[0]).handle, p, len(data), int(skipword),
                                        ctypes.byref(out)), "pnetgpu_util_checksum")
        return int(out.value)

    @staticmethod
    def _pseudo(version, data, skipword, extra_data, source, destination, next_level_protocol):
        ctypes, lib = _host_setup()
        from ._lib import check
        alen = 4 if version == 4 else 16
        data, p = util_host._buf(data)
        extra, e = util_host._buf(extra_data or b"")
        s, d = _addr(source, alen), _addr(destination, alen)
        fn = lib.pnetgpu_util_ipv4_checksum if version == 4 else lib.pnetgpu_util_ipv6_checksum
        out = ctypes.c_uint16()
        check(fn(engine.context(_DEVICE[0]).handle, p, len(data), int(skipword), e, len(extra), s, d,
                 int(next_level_protocol) & 0xFF, ctypes.byref(out)), f"pnetgpu_util_ipv{version}_checksum")
        return int(out.value)

    @staticmethod
    def ipv4_checksum(data, skipword, extra_data, source, destination, next_level_protocol):
        return util_host._pseudo(4, data, skipword, extra_data, source, destination, next_level_protocol)

    @staticmethod
    def ipv6_checksum(data, skipword, extra_data, source, destination, next_level_protocol):
        return util_host._pseudo(6, data, skipword, extra_data, source, destination, next_level_protocol)

    @staticmethod
    def checksum_slices(buf, offsets, lengths, skipwords):
        """pnetgpu_checksum_slices_host over host numpy arrays; returns uint16 words."""
        ctypes, lib = _host_setup()
        from ._lib import check
        buf = np.ascontiguousarray(buf, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        lengths = np.ascontiguousarray(lengths, np.uint32)
        skipwords = np.ascontiguousarray(skipwords, np.uint32)
        n = len(offsets)
        out = np.zeros(n, np.uint16)
        check(lib.pnetgpu_checksum_slices_host(engine.context(_DEVICE[0]).handle, buf.ctypes.data, buf.size, n,
                                               offsets.ctypes.data, lengths.ctypes.data, skipwords.ctypes.data,
                                               out.ctypes.data), "pnetgpu_checksum_slices_host")
        return out
