"""Synthetic BASELINE.json workloads from the native producer (include/pnetgpu_synth.h)."""
import ctypes
import os

import numpy as np

from ._lib import DEFS, check, lib

WORKLOADS = {
    "rs_sender": DEFS["PNETGPU_SYNTH_RS_SENDER"],
    "udp64": DEFS["PNETGPU_SYNTH_UDP64"],
    "tcp1500": DEFS["PNETGPU_SYNTH_TCP1500"],
    "udp1500": DEFS["PNETGPU_SYNTH_UDP1500"],
    "imix": DEFS["PNETGPU_SYNTH_IMIX"],
    "udp6_jumbo": DEFS["PNETGPU_SYNTH_UDP6_JUMBO"],
}


class Workload:
    """Host-side frame batch: buf (uint8), offsets/lengths (descriptor mode) or stride."""

    def __init__(self, name, n, buf, stride, frame_len, offsets, lengths, expect):
        self.name, self.n, self.buf = name, n, buf
        self.stride, self.frame_len = stride, frame_len
        self.offsets, self.lengths = offsets, lengths
        self.expect = {"ip_bad": int(expect[0]), "l4_bad": int(expect[1]), "bytes": int(expect[2])}


def layout(name, n, seed=0, first=0):
    tot, st, fl = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
    check(lib.pnetgpu_synth_layout_range(WORKLOADS[name], first, n, seed, ctypes.byref(tot), ctypes.byref(st),
                                         ctypes.byref(fl)), "pnetgpu_synth_layout_range")
    return tot.value, st.value, fl.value


def lengths(name, n, seed=0, first=0):
    """Frame lengths of frames [first, first + n) of a workload's batch (nothing built)."""
    out = np.empty(n, dtype=np.uint32)
    check(lib.pnetgpu_synth_lengths(WORKLOADS[name], first, n, seed, ctypes.c_void_p(out.ctypes.data)),
          "pnetgpu_synth_lengths")
    return out


def make(name, n, seed=0, corrupt_ppm=10000, nthreads=None, buf=None, first=0):
    """Build n frames of a workload: frames [first, first + n) of the batch `seed`
    defines (a shard of a global batch, byte-identical to those frames of the
    whole batch). `buf` may be a preallocated (e.g. pinned) uint8 array/tensor."""
    total, stride, flen = layout(name, n, seed, first)
    if buf is None:
        buf = np.empty(total, dtype=np.uint8)
    addr = buf.ctypes.data if isinstance(buf, np.ndarray) else buf.data_ptr()
    size = buf.size if isinstance(buf, np.ndarray) else buf.numel()
    offsets = lengths = None
    if stride == 0:
        offsets = np.empty(n, dtype=np.uint64)
        lengths = np.empty(n, dtype=np.uint32)
    exp = (ctypes.c_uint64 * 3)()
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    check(lib.pnetgpu_synth_fill_range(WORKLOADS[name], first, n, seed, corrupt_ppm, ctypes.c_void_p(addr), size,
                                       ctypes.c_void_p(offsets.ctypes.data if offsets is not None else 0),
                                       ctypes.c_void_p(lengths.ctypes.data if lengths is not None else 0),
                                       exp, nthreads), "pnetgpu_synth_fill_range")
    return Workload(name, n, buf, stride, flen, offsets, lengths, list(exp))
