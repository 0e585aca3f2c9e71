"""ctypes binding of libpnetgpu.so (include/pnetgpu.h, include/pnetgpu_synth.h).

The in-tree shared library is the only implementation: if it is missing or
fails to load, importing libpnet_amd raises — there is no CPU fallback.
"""
import ctypes
import os
import re

# PyTorch-ROCm bundles its own libamdhip64.so.7. Import it first so that the
# dynamic loader resolves libpnetgpu.so's libamdhip64.so.7 (same SONAME) to the
# runtime already in the process: one HIP runtime, shared device pointers/streams.
import torch  # noqa: F401

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
# PNETGPU_LIB selects an alternative build of the same library (tuning A/B runs)
LIB_PATH = os.environ.get("PNETGPU_LIB") or os.path.join(PKG_DIR, "libpnetgpu.so")
HEADERS = [os.path.join(ROOT, "include", h)
           for h in ("pnetgpu.h", "pnetgpu_synth.h", "pnetgpu_ring.h", "pnetgpu_afpacket.h", "pnetgpu_util.h")]


class PnetGpuError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = _lib.pnetgpu_strerror(code).decode() if _lib is not None else str(code)
        self.hip_error = _lib.pnetgpu_last_hip_error() if _lib is not None and code == -3 else 0
        if self.hip_error:
            msg += f", hipError_t {self.hip_error}"
        super().__init__(f"{what}: pnetgpu error {code} ({msg})")


def _header_defines():
    """Integer #define constants of the public headers (the ABI's numbers)."""
    out = {}
    for h in HEADERS:
        with open(h) as fh:
            for line in fh:
                m = re.match(r"#define\s+(P[A-Z0-9_]+)\s+([^/]+?)\s*(/\*.*)?$", line)
                if not m:
                    continue
                expr = re.sub(r"\b(0[xX][0-9a-fA-F]+|\d+)[uU]\b", r"\1", m.group(2))
                if not re.fullmatch(r"[\w\s()<>|+-]+", expr):
                    continue
                try:
                    out[m.group(1)] = int(eval(expr, {"__builtins__": {}}, dict(out)))
                except Exception:
                    pass
    return out


DEFS = _header_defines()


class Batch(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("data_bytes", ctypes.c_uint64), ("n_frames", ctypes.c_uint64),
                ("first_offset", ctypes.c_uint64), ("stride", ctypes.c_uint32), ("frame_len", ctypes.c_uint32),
                ("offsets", ctypes.c_void_p), ("lengths", ctypes.c_void_p), ("flags", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class SliceDesc(ctypes.Structure):
    """pnetgpu_slice_desc: the compact (8-B) slice descriptor."""
    _fields_ = [("offset", ctypes.c_uint32), ("length", ctypes.c_uint16), ("skipword", ctypes.c_uint16)]


# pnetgpu_rx_columns in struct order: the record columns, `counters`, then the
# header-field columns of ABI v3
COLUMN_NAMES = ("status", "ip_csum", "l4_csum", "ethertype", "ip_proto", "ttl", "l4_offset", "l4_length",
                "src_port", "dst_port", "src_ipv4", "dst_ipv4", "src_ipv6", "dst_ipv6", "vlan_tci", "l3_offset")
FIELD_COLUMN_NAMES = ("eth_dst", "eth_src", "ip_version", "ip_header_length", "ip_dscp", "ip_ecn", "ip_total_length",
                      "ip_identification", "ip_flags", "ip_fragment_offset", "ip6_traffic_class", "ip6_flow_label",
                      "ip6_payload_length", "udp_length", "tcp_sequence", "tcp_acknowledgement", "tcp_data_offset",
                      "tcp_reserved", "tcp_flags", "tcp_window", "tcp_urgent_ptr", "icmp_sequence")
ALL_COLUMN_NAMES = COLUMN_NAMES + FIELD_COLUMN_NAMES


class RxColumns(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_void_p) for n in COLUMN_NAMES] + [("counters", ctypes.c_void_p)]
                + [(n, ctypes.c_void_p) for n in FIELD_COLUMN_NAMES])


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libpnet_amd: native library {LIB_PATH} is not built "
                          "(run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C libpnet_amd`)")
    L = ctypes.CDLL(LIB_PATH, use_errno=True)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.pnetgpu_abi_version.restype = i32
    L.pnetgpu_strerror.restype = ctypes.c_char_p
    L.pnetgpu_strerror.argtypes = [i32]
    L.pnetgpu_last_hip_error.restype = i32
    L.pnetgpu_last_hip_error.argtypes = []
    L.pnetgpu_last_rx_kernel.restype = ctypes.c_char_p
    L.pnetgpu_last_rx_kernel.argtypes = []
    L.pnetgpu_device_count.restype = i32
    L.pnetgpu_device_count.argtypes = [ctypes.POINTER(i32)]
    L.pnetgpu_ctx_create.restype = i32
    L.pnetgpu_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.pnetgpu_ctx_destroy.restype = None
    L.pnetgpu_ctx_destroy.argtypes = [vp]
    L.pnetgpu_ctx_set_tuning.restype = i32
    L.pnetgpu_ctx_set_tuning.argtypes = [vp, i32, ctypes.c_int64]
    L.pnetgpu_ctx_get_tuning.restype = i32
    L.pnetgpu_ctx_get_tuning.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_int64)]
    L.pnetgpu_ctx_sched_conflicts.restype = i32
    L.pnetgpu_ctx_sched_conflicts.argtypes = [vp, ctypes.POINTER(u64)]
    L.pnetgpu_desc_size_hint.restype = u32
    L.pnetgpu_desc_size_hint.argtypes = [vp, u64]
    L.pnetgpu_ctx_sched_stats.restype = i32
    L.pnetgpu_ctx_sched_stats.argtypes = [vp, vp]
    for f in (L.pnetgpu_rx_process, L.pnetgpu_tx_fill_checksums):
        f.restype = i32
        f.argtypes = [vp, ctypes.POINTER(Batch), ctypes.POINTER(RxColumns), vp]
    L.pnetgpu_checksum_slices.restype = i32
    L.pnetgpu_checksum_slices.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp, vp]
    L.pnetgpu_checksum_slices_compact.restype = i32
    L.pnetgpu_checksum_slices_compact.argtypes = [vp, vp, u64, u64, vp, vp, vp]
    L.pnetgpu_checksum_slices_strided.restype = i32
    L.pnetgpu_checksum_slices_strided.argtypes = [vp, vp, u64, u64, u64, u32, u32, u32, vp, vp]
    for f in (L.pnetgpu_ipv4_checksum_slices, L.pnetgpu_ipv6_checksum_slices):
        f.restype = i32
        f.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, vp]
    for f in (L.pnetgpu_ipv4_checksum_adv_slices, L.pnetgpu_ipv6_checksum_adv_slices):
        f.restype = i32
        f.argtypes = [vp, vp, u64, u64, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.pnetgpu_synth_layout.restype = i32
    L.pnetgpu_synth_layout.argtypes = [i32, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u32),
                                       ctypes.POINTER(u32)]
    L.pnetgpu_synth_fill.restype = i32
    L.pnetgpu_synth_fill.argtypes = [i32, u64, u64, u32, vp, u64, vp, vp, vp, i32]
    L.pnetgpu_synth_layout_range.restype = i32
    L.pnetgpu_synth_layout_range.argtypes = [i32, u64, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u32),
                                             ctypes.POINTER(u32)]
    L.pnetgpu_synth_fill_range.restype = i32
    L.pnetgpu_synth_fill_range.argtypes = [i32, u64, u64, u64, u32, vp, u64, vp, vp, vp, i32]
    L.pnetgpu_synth_lengths.restype = i32
    L.pnetgpu_synth_lengths.argtypes = [i32, u64, u64, u64, vp]
    if L.pnetgpu_abi_version() != DEFS["PNETGPU_ABI_VERSION"]:
        raise ImportError("libpnet_amd: libpnetgpu.so ABI version does not match include/pnetgpu.h")
    return L


_lib = None
_lib = _load()
lib = _lib


def check(rc, what):
    if rc != 0:
        raise PnetGpuError(rc, what)
