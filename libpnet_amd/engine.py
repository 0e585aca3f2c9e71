"""Host-side engine over the C-ABI: the batched receive path and batched checksums.

Mirrors the reference's operator surface for this path:

  rx_process(...)            — the per-frame chain packetdump.rs:120-217 runs
                               (EthernetPacket::new → Ipv4/Ipv6Packet::new →
                               ipv4::checksum → payload() → Udp/Tcp/IcmpPacket::new →
                               udp/tcp::ipv4_checksum|ipv6_checksum, icmp(v6)::checksum),
                               for a whole device-resident batch at once.
  checksum_slices(...)       — pnet_packet::util::checksum           (util.rs:76-82)
  ipv4_checksum_slices(...)  — pnet_packet::util::ipv4_checksum      (util.rs:92-117)
  ipv6_checksum_slices(...)  — pnet_packet::util::ipv6_checksum      (util.rs:125-150)

Device memory and streams come from PyTorch (plumbing only); all compute is the
HIP kernels of libpnetgpu.so. Unsigned columns are stored in signed torch dtypes
of the same width; RxResult.numpy() returns the unsigned views.
"""
import ctypes
from contextlib import contextmanager
from contextlib import nullcontext as _nullcontext

import numpy as np
import torch

from ._lib import ALL_COLUMN_NAMES, COLUMN_NAMES, DEFS, FIELD_COLUMN_NAMES, Batch, RxColumns, check, lib

# column -> (torch storage dtype, numpy view dtype, trailing shape)
COLUMNS = {
    "status": (torch.int16, np.uint16, ()),
    "ip_csum": (torch.int16, np.uint16, ()),
    "l4_csum": (torch.int16, np.uint16, ()),
    "ethertype": (torch.int16, np.uint16, ()),
    "ip_proto": (torch.uint8, np.uint8, ()),
    "ttl": (torch.uint8, np.uint8, ()),
    "l4_offset": (torch.int16, np.uint16, ()),
    "l4_length": (torch.int16, np.uint16, ()),
    "src_port": (torch.int16, np.uint16, ()),
    "dst_port": (torch.int16, np.uint16, ()),
    "src_ipv4": (torch.int32, np.uint32, ()),
    "dst_ipv4": (torch.int32, np.uint32, ()),
    "src_ipv6": (torch.uint8, np.uint8, (16,)),
    "dst_ipv6": (torch.uint8, np.uint8, (16,)),
    "vlan_tci": (torch.int16, np.uint16, ()),
    "l3_offset": (torch.uint8, np.uint8, ()),
    # header-field columns (ABI v3): the remaining generated getters
    "eth_dst": (torch.int64, np.uint64, ()),
    "eth_src": (torch.int64, np.uint64, ()),
    "ip_version": (torch.uint8, np.uint8, ()),
    "ip_header_length": (torch.uint8, np.uint8, ()),
    "ip_dscp": (torch.uint8, np.uint8, ()),
    "ip_ecn": (torch.uint8, np.uint8, ()),
    "ip_total_length": (torch.int16, np.uint16, ()),
    "ip_identification": (torch.int16, np.uint16, ()),
    "ip_flags": (torch.uint8, np.uint8, ()),
    "ip_fragment_offset": (torch.int16, np.uint16, ()),
    "ip6_traffic_class": (torch.uint8, np.uint8, ()),
    "ip6_flow_label": (torch.int32, np.uint32, ()),
    "ip6_payload_length": (torch.int16, np.uint16, ()),
    "udp_length": (torch.int16, np.uint16, ()),
    "tcp_sequence": (torch.int32, np.uint32, ()),
    "tcp_acknowledgement": (torch.int32, np.uint32, ()),
    "tcp_data_offset": (torch.uint8, np.uint8, ()),
    "tcp_reserved": (torch.uint8, np.uint8, ()),
    "tcp_flags": (torch.uint8, np.uint8, ()),
    "tcp_window": (torch.int16, np.uint16, ()),
    "tcp_urgent_ptr": (torch.int16, np.uint16, ()),
    "icmp_sequence": (torch.int16, np.uint16, ()),
}
assert tuple(COLUMNS) == ALL_COLUMN_NAMES

#: every IPv4-relevant column: the bench's "checksum verify + header extract" record
IPV4_COLUMNS = ("status", "ip_csum", "l4_csum", "ethertype", "ip_proto", "ttl", "l4_offset", "l4_length",
                "src_port", "dst_port", "src_ipv4", "dst_ipv4")
RX_VLAN, RX_IPV6_EXT, RX_L3 = DEFS["PNETGPU_RX_VLAN"], DEFS["PNETGPU_RX_IPV6_EXT"], DEFS["PNETGPU_RX_L3"]
DESC_COMPACT = DEFS["PNETGPU_DESC_COMPACT"]
#: frame-size hints of a descriptor batch (the tail shape only; records are identical)
DESC_HINT_LARGE, DESC_HINT_JUMBO = DEFS["PNETGPU_DESC_HINT_LARGE"], DEFS["PNETGPU_DESC_HINT_JUMBO"]


def desc_size_hint(lengths):
    """pnetgpu_desc_size_hint over host-side frame lengths: DESC_HINT_JUMBO,
    DESC_HINT_LARGE or 0, to OR into rx_process's flags for a descriptor batch."""
    a = np.ascontiguousarray(lengths, dtype=np.uint32)
    return int(lib.pnetgpu_desc_size_hint(ctypes.c_void_p(a.ctypes.data), a.size))
#: every column: the record columns and the ABI-v3 header-field getters
ALL_COLUMNS = ALL_COLUMN_NAMES
#: the record columns of ABI v2 (status, checksums, dispatch fields, addresses, VLAN, L3 offset)
RECORD_COLUMNS = COLUMN_NAMES
#: the header-field getter columns (eth MACs, IPv4/IPv6 header fields, UDP length, TCP header, ICMP echo sequence)
FIELD_COLUMNS = FIELD_COLUMN_NAMES
NCOUNTERS = DEFS["PNETGPU_NCOUNTERS"]
COUNTER_NAMES = ("frames", "bytes", "ipv4", "ipv6", "ip_csum_bad", "l4_csum_bad", "malformed", "unknown")


def column_bytes(columns):
    """Result bytes written per frame for a column set (the R of the roofline)."""
    out = 0
    for c in columns:
        dt, npdt, shape = COLUMNS[c]
        out += np.dtype(npdt).itemsize * int(np.prod(shape or (1,)))
    return out


#: tuning keys of pnetgpu_ctx_set_tuning (PNETGPU_TUNE_<NAME>), by lower-case name
TUNING_KEYS = {k[len("PNETGPU_TUNE_"):].lower(): v for k, v in DEFS.items() if k.startswith("PNETGPU_TUNE_")}
_SLICE_KERNELS = {"run": 1, "group": 2, "tiny": 3}


class Context:
    """One pnetgpu_ctx bound to a HIP device."""

    def __init__(self, device=0):
        self.device = int(device)
        h = ctypes.c_void_p()
        check(lib.pnetgpu_ctx_create(self.device, ctypes.byref(h)), "pnetgpu_ctx_create")
        self.handle = h

    def set_tuning(self, name, value):
        """pnetgpu_ctx_set_tuning: override a kernel default on this context
        (name: a TUNING_KEYS key, e.g. "static_pct"; value None or -1 restores
        the default; slice_kernel also takes "run" / "group" / "tiny")."""
        if name not in TUNING_KEYS:
            raise KeyError(f"unknown tuning key {name!r} (one of {sorted(TUNING_KEYS)})")
        v = -1 if value is None else _SLICE_KERNELS.get(value, value)
        check(lib.pnetgpu_ctx_set_tuning(self.handle, TUNING_KEYS[name], int(v)), f"set_tuning({name}={value})")

    def get_tuning(self, name):
        """The current setting (-1: the default)."""
        v = ctypes.c_int64()
        check(lib.pnetgpu_ctx_get_tuning(self.handle, TUNING_KEYS[name], ctypes.byref(v)), "get_tuning")
        return v.value

    @contextmanager
    def tuning(self, **settings):
        """Apply settings for the duration of a with-block, then restore them."""
        old = {k: self.get_tuning(k) for k in settings}
        try:
            for k, v in settings.items():
                self.set_tuning(k, v)
            yield self
        finally:
            for k, v in old.items():
                self.set_tuning(k, v)

    def sched_conflicts(self):
        """pnetgpu_ctx_sched_conflicts: always 0 (launches never share claim counters)."""
        v = ctypes.c_uint64()
        check(lib.pnetgpu_ctx_sched_conflicts(self.handle, ctypes.byref(v)), "pnetgpu_ctx_sched_conflicts")
        return v.value

    def sched_stats(self):
        """pnetgpu_ctx_sched_stats: {"claimed", "static_busy", "static_captured",
        "blocks_held", "blocks"} — launches that took a counter block, ran static
        because every block was held, or were captured into a graph; blocks
        held now and the pool size."""
        v = (ctypes.c_uint64 * DEFS["PNETGPU_NSCHED_STATS"])()
        check(lib.pnetgpu_ctx_sched_stats(self.handle, v), "pnetgpu_ctx_sched_stats")
        return dict(zip(("claimed", "static_busy", "static_captured", "blocks_held", "blocks"), (int(x) for x in v)))

    def close(self):
        if getattr(self, "handle", None):
            lib.pnetgpu_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts = {}


def context(device=None):
    if device is None:
        device = torch.cuda.current_device()
    if isinstance(device, torch.device):
        device = device.index or 0
    elif isinstance(device, str):
        device = torch.device(device).index or 0
    if device not in _contexts:
        _contexts[device] = Context(device)
    return _contexts[device]


def tuning(device=None, **settings):
    """Context manager: tuning settings on the shared context of `device`
    (Context.tuning), e.g. `with engine.tuning(static_pct=0, claim_counters=4):`."""
    return context(device).tuning(**settings)


def apply_tuning_env(settings, device=None):
    """Measurement tools: apply {"PNETGPU_<NAME>": value} settings (named as the
    environment variables a context reads at creation) to the shared context of
    `device` through pnetgpu_ctx_set_tuning; "" or None restores the default."""
    ctx = context(device)
    for k, v in settings.items():
        name = k[len("PNETGPU_"):].lower() if k.startswith("PNETGPU_") else k
        if v in ("", None):
            ctx.set_tuning(name, None)
        else:
            ctx.set_tuning(name, v if name == "slice_kernel" and v in _SLICE_KERNELS else int(v))


def _stream_handle(stream, device):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class RxResult:
    """Device-resident result columns of one rx_process call, packed back to back
    (each 256-B aligned) in one allocation, `block`: the counters first, then
    the columns, so the whole record moves to the host in one copy (to_host)."""

    def __init__(self, n, device, columns=IPV4_COLUMNS, counters=True):
        self.n = n
        layout, at = [], 8 * NCOUNTERS if counters else 0
        for c in columns:
            dt, _, shape = COLUMNS[c]
            at = (at + 255) & ~255
            nbytes = n * int(np.prod(shape, dtype=np.int64)) * torch.empty((), dtype=dt).element_size()
            layout.append((c, at, nbytes, dt, shape))
            at += nbytes
        self.block = torch.empty(max(at, 1), dtype=torch.uint8, device=device)
        self.columns = {c: self.block[o:o + nb].view(dt).view((n,) + shape) for c, o, nb, dt, shape in layout}
        self.counters = None
        if counters:
            self.counters = self.block[:8 * NCOUNTERS].view(torch.int64)
            self.counters.zero_()
        self.nbytes = at

    def to_host(self, out=None, stream=None):
        """Copy counters + columns to host memory in one D2H (out: a pinned
        uint8 tensor of at least nbytes, or None for a new one); returns out."""
        if out is None:
            out = torch.empty(self.nbytes, dtype=torch.uint8).pin_memory()
        with torch.cuda.stream(stream) if stream is not None else _nullcontext():
            out[:self.nbytes].copy_(self.block[:self.nbytes], non_blocking=True)
        return out

    def c_struct(self):
        cols = RxColumns()
        for c in ALL_COLUMN_NAMES:
            setattr(cols, c, self.columns[c].data_ptr() if c in self.columns else 0)
        cols.counters = self.counters.data_ptr() if self.counters is not None else 0
        return cols

    def numpy(self):
        """Every column as an unsigned numpy array (one D2H copy of the block)."""
        h = self.block[:self.nbytes].cpu().numpy() if self.block.is_cuda else self.block[:self.nbytes].numpy()
        base = self.block.data_ptr()
        out = {}
        for c, t in self.columns.items():
            o = t.data_ptr() - base
            nb = t.numel() * t.element_size()
            out[c] = h[o:o + nb].view(COLUMNS[c][1]).reshape(tuple(t.shape))
        return out

    def counter_dict(self):
        if self.counters is None:
            return {}
        v = self.counters.cpu().numpy().view(np.uint64)
        return dict(zip(COUNTER_NAMES, (int(x) for x in v)))


def _check_u8_cuda(t, what):
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.uint8 and t.is_contiguous()):
        raise TypeError(f"{what} must be a contiguous torch.uint8 CUDA tensor")


def _check_dev(t, what, dtypes, device, numel):
    """A device array the kernels read: contiguous, of one of `dtypes`, on the
    data's device and holding at least `numel` elements (a host pointer or a
    short array would fault the GPU or read past the end)."""
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.device == device and t.is_contiguous()):
        raise TypeError(f"{what} must be a contiguous CUDA tensor on {device}")
    if t.dtype not in dtypes:
        raise TypeError(f"{what} must be one of {[str(d) for d in dtypes]}, not {t.dtype}")
    if t.numel() < numel:
        raise ValueError(f"{what} holds {t.numel()} elements, {numel} needed")


_I64, _I32, _U8 = (torch.int64, torch.uint64), (torch.int32, torch.uint32), (torch.uint8,)


def last_rx_kernel():
    """The kernel instantiation the calling thread's last rx_process /
    tx_fill_checksums / *_slices call launched, named as rocprofv3 names it
    (pnetgpu_last_rx_kernel)."""
    return lib.pnetgpu_last_rx_kernel().decode()


def rx_process(data, *, n_frames=None, stride=0, frame_len=None, first_offset=0, offsets=None, lengths=None,
               columns=IPV4_COLUMNS, counters=True, out=None, stream=None, data_bytes=None, flags=0, ctx=None):
    """Parse + verify every frame of a device-resident batch.

    Fixed-stride mode: stride > 0, frame i = data[first_offset + i*stride, +frame_len).
    Descriptor mode:   offsets (int64) / lengths (int32) CUDA tensors, frame i = data[off_i, +len_i);
                       with flags |= DESC_COMPACT, offsets (u32 as int32/uint32) / lengths
                       (u16 as int16/uint16) — 6 B per frame of descriptors instead of 12;
                       flags |= desc_size_hint(host_lengths) names the kernel's tail
                       shape for the batch's size mix (MTU / jumbo frames).
    ctx: a Context (default: one shared per device); one host thread per context at a time.
    Returns an RxResult (device columns, accumulated counters)."""
    return _rx_or_tx("pnetgpu_rx_process", data, n_frames, stride, frame_len, first_offset, offsets, lengths,
                     columns, counters, out, stream, data_bytes, flags, ctx)


def tx_fill_checksums(data, *, n_frames=None, stride=0, frame_len=None, first_offset=0, offsets=None,
                      lengths=None, columns=("status",), counters=False, out=None, stream=None, data_bytes=None,
                      flags=0):
    """Sender side: write every checksum the receive path computes into its field, in place
    (set_checksum(ipv4::checksum(..)), set_checksum(udp::ipv4_checksum(..)), ... as
    benches/rs_sender.rs:38-39,70-71). Frames must not overlap. The returned columns
    describe the frames before patching."""
    return _rx_or_tx("pnetgpu_tx_fill_checksums", data, n_frames, stride, frame_len, first_offset, offsets,
                     lengths, columns, counters, out, stream, data_bytes, flags)


def _rx_or_tx(fn_name, data, n_frames, stride, frame_len, first_offset, offsets, lengths, columns, counters, out,
              stream, data_bytes, flags, ctx=None):
    _check_u8_cuda(data, "data")
    if stride:
        if n_frames is None:
            n_frames = (data.numel() - first_offset) // stride
        if frame_len is None:
            frame_len = stride
    else:
        if offsets is None or lengths is None:
            raise ValueError("descriptor mode needs offsets and lengths")
        for t, what in ((offsets, "offsets"), (lengths, "lengths")):
            if not (isinstance(t, torch.Tensor) and t.is_cuda and t.device == data.device and t.is_contiguous()):
                raise TypeError(f"{what} must be a contiguous CUDA tensor on {data.device}")
        if flags & DESC_COMPACT:
            if offsets.dtype not in (torch.int32, torch.uint32) or lengths.dtype not in (torch.int16, torch.uint16):
                raise TypeError("DESC_COMPACT: offsets must be 32-bit and lengths 16-bit CUDA tensors")
        elif offsets.dtype != torch.int64 or lengths.dtype != torch.int32:
            raise TypeError("offsets must be int64 and lengths int32 CUDA tensors")
        if n_frames is None:
            n_frames = offsets.numel()
        if not 0 <= n_frames <= min(offsets.numel(), lengths.numel()):
            raise ValueError(f"n_frames={n_frames} exceeds the descriptors ({offsets.numel()} offsets, "
                             f"{lengths.numel()} lengths)")
        frame_len = 0
    if out is None:
        out = RxResult(n_frames, data.device, columns, counters)
    elif out.n < n_frames:
        raise ValueError(f"out holds {out.n} frames, the batch has {n_frames}")
    b = Batch(data.data_ptr(), data.numel() if data_bytes is None else data_bytes, n_frames, first_offset,
              stride, frame_len, offsets.data_ptr() if offsets is not None else 0,
              lengths.data_ptr() if lengths is not None else 0, flags, 0)
    cols = out.c_struct()
    if ctx is None:
        ctx = context(data.device.index)
    check(getattr(lib, fn_name)(ctx.handle, ctypes.byref(b), ctypes.byref(cols),
                                _stream_handle(stream, data.device)), fn_name)
    return out


def _slices(fn_name, data, offsets, lengths, skipwords, addrs=None, protos=None, stream=None, alen=0):
    _check_u8_cuda(data, "data")
    n = offsets.numel()
    _check_dev(offsets, "offsets", _I64, data.device, n)
    _check_dev(lengths, "lengths", _I32, data.device, n)
    _check_dev(skipwords, "skipwords", _I32, data.device, n)
    if addrs is not None:
        _check_dev(addrs, "addrs", _U8, data.device, n * alen)
        _check_dev(protos, "protos", _U8, data.device, n)
    out = torch.empty(n, dtype=torch.int16, device=data.device)
    ctx = context(data.device.index)
    args = [ctx.handle, _ptr(data), data.numel(), n, _ptr(offsets), _ptr(lengths), _ptr(skipwords)]
    if addrs is not None:
        args += [_ptr(addrs), _ptr(protos)]
    args += [_ptr(out), _stream_handle(stream, data.device)]
    check(getattr(lib, fn_name)(*args), fn_name)
    return out


def checksum_slices(data, offsets, lengths, skipwords, stream=None):
    """out[i] = util::checksum(data[off_i, +len_i), skipwords[i]) (uint16 in an int16 tensor)."""
    return _slices("pnetgpu_checksum_slices", data, offsets, lengths, skipwords, stream=stream)


def slice_descriptors(offsets, lengths, skipwords, device=None):
    """Pack (offset, length, skipword) triples into compact pnetgpu_slice_desc
    records (u32, u16, u16 = 8 B each) as an int64 tensor (on `device` if given)."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    lengths = np.asarray(lengths, dtype=np.uint64)
    skipwords = np.asarray(skipwords, dtype=np.uint64)
    if offsets.size and (offsets.max() > 0xFFFFFFFF or lengths.max() > 0xFFFF or skipwords.max() > 0xFFFF):
        raise ValueError("compact slice descriptors need offsets < 2^32, lengths and skipwords < 2^16")
    packed = offsets | (lengths << np.uint64(32)) | (skipwords << np.uint64(48))
    t = torch.from_numpy(packed.view(np.int64))
    return t.to(device) if device is not None else t


def checksum_slices_compact(data, desc, stream=None):
    """out[i] = util::checksum over compact descriptors (slice_descriptors(...)):
    pnetgpu_checksum_slices_compact. Descriptors held elsewhere than the data's
    device (e.g. slice_descriptors' host tensor) are copied there first."""
    _check_u8_cuda(data, "data")
    if not isinstance(desc, torch.Tensor) or desc.dtype not in _I64:
        raise TypeError("desc must be an int64 / uint64 tensor of packed pnetgpu_slice_desc records")
    copied = not desc.is_cuda or desc.device != data.device or not desc.is_contiguous()
    with torch.cuda.stream(stream) if stream is not None else _nullcontext():
        # the copy (and the output) on the launch's stream: ordered before the
        # kernel, and the allocator's stream for the temporary is the one that reads it
        if copied:
            desc = desc.to(data.device).contiguous()
        n = desc.numel()
        out = torch.empty(n, dtype=torch.int16, device=data.device)
    ctx = context(data.device.index)
    check(lib.pnetgpu_checksum_slices_compact(ctx.handle, _ptr(data), data.numel(), n, _ptr(desc), _ptr(out),
                                              _stream_handle(stream, data.device)), "pnetgpu_checksum_slices_compact")
    return out


def checksum_slices_strided(data, n, stride, slice_len, skipword, first_offset=0, stream=None):
    """out[i] = util::checksum(data[first_offset + i*stride, +slice_len), skipword), i < n:
    uniform slices without descriptor arrays (pnetgpu_checksum_slices_strided)."""
    _check_u8_cuda(data, "data")
    for v, what in ((stride, "stride"), (slice_len, "slice_len"), (skipword, "skipword")):
        if not 0 <= int(v) < (1 << 32):   # u32 in the C-ABI: never truncated
            raise ValueError(f"{what}={v} must be in [0, 2^32)")
    if int(n) < 0 or int(first_offset) < 0:
        raise ValueError("n and first_offset must be non-negative")
    out = torch.empty(n, dtype=torch.int16, device=data.device)
    ctx = context(data.device.index)
    check(lib.pnetgpu_checksum_slices_strided(ctx.handle, _ptr(data), data.numel(), n, first_offset, stride,
                                              slice_len, skipword, _ptr(out), _stream_handle(stream, data.device)),
          "pnetgpu_checksum_slices_strided")
    return out


def ipv4_checksum_slices(data, offsets, lengths, skipwords, addrs, protos, stream=None):
    """util::ipv4_checksum per slice; addrs uint8 [n, 8] (src||dst), protos uint8 [n]."""
    return _slices("pnetgpu_ipv4_checksum_slices", data, offsets, lengths, skipwords, addrs, protos, stream, alen=8)


def checksum_adv_slices(version, data, offsets, lengths, skipwords, extra_offsets, extra_lengths, addrs, protos,
                        stream=None):
    """util::ipv4_checksum / ipv6_checksum with extra_data (the *_checksum_adv wrappers):
    version 4 (addrs [n, 8]) or 6 (addrs [n, 32])."""
    _check_u8_cuda(data, "data")
    n = offsets.numel()
    for t, what, dts, k in ((offsets, "offsets", _I64, 1), (lengths, "lengths", _I32, 1),
                            (skipwords, "skipwords", _I32, 1), (extra_offsets, "extra_offsets", _I64, 1),
                            (extra_lengths, "extra_lengths", _I32, 1), (addrs, "addrs", _U8, 8 if version == 4 else 32),
                            (protos, "protos", _U8, 1)):
        _check_dev(t, what, dts, data.device, n * k)
    out = torch.empty(n, dtype=torch.int16, device=data.device)
    ctx = context(data.device.index)
    fn = "pnetgpu_ipv4_checksum_adv_slices" if version == 4 else "pnetgpu_ipv6_checksum_adv_slices"
    check(getattr(lib, fn)(ctx.handle, _ptr(data), data.numel(), n, _ptr(offsets), _ptr(lengths), _ptr(skipwords),
                           _ptr(extra_offsets), _ptr(extra_lengths), _ptr(addrs), _ptr(protos), _ptr(out),
                           _stream_handle(stream, data.device)), fn)
    return out


def ipv6_checksum_slices(data, offsets, lengths, skipwords, addrs, protos, stream=None):
    """util::ipv6_checksum per slice; addrs uint8 [n, 32] (src||dst), protos uint8 [n]."""
    return _slices("pnetgpu_ipv6_checksum_slices", data, offsets, lengths, skipwords, addrs, protos, stream, alen=32)
