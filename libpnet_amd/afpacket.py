"""AF_PACKET TPACKET_V3 receive ring as a batch producer (include/pnetgpu_afpacket.h):
the pnet_datalink Linux receiver (pnet_datalink/src/linux.rs:362-403) as a mapped
block ring whose retired blocks are shipped zero-copy through Ring.feed_region."""
import ctypes

import numpy as np

from ._lib import PnetGpuError, check, lib

ESYS, EEMPTY = -9, -7
TP_STATUS_CSUMNOTREADY = 1 << 3

_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
lib.pnetgpu_afp_open.restype = ctypes.c_int32
lib.pnetgpu_afp_open.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                 ctypes.POINTER(ctypes.c_void_p)]
lib.pnetgpu_afp_close.restype = None
lib.pnetgpu_afp_close.argtypes = [ctypes.c_void_p]
lib.pnetgpu_afp_ring.restype = ctypes.c_int32
lib.pnetgpu_afp_ring.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), _u64p, _u32p, _u32p]
lib.pnetgpu_afp_next_block.restype = ctypes.c_int32
lib.pnetgpu_afp_next_block.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_uint64, _u64p, _u32p]
lib.pnetgpu_afp_release_block.restype = ctypes.c_int32
lib.pnetgpu_afp_release_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
lib.pnetgpu_afp_stats.restype = ctypes.c_int32
lib.pnetgpu_afp_stats.argtypes = [ctypes.c_void_p, _u64p, _u64p]
lib.pnetgpu_afp_fanout.restype = ctypes.c_int32
lib.pnetgpu_afp_fanout.argtypes = [ctypes.c_void_p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32]
lib.pnetgpu_afp_promiscuous.restype = ctypes.c_int32
lib.pnetgpu_afp_promiscuous.argtypes = [ctypes.c_void_p, ctypes.c_int]
FANOUT = {"hash": 0, "lb": 1, "cpu": 2, "rollover": 3, "rnd": 4, "qm": 5}
lib.pnetgpu_tpacket3_walk.restype = ctypes.c_int32
lib.pnetgpu_tpacket3_walk.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, _u64p]


def tpacket3_walk(block, block_offset=0, cap=1 << 16):
    """(offsets uint64, lengths uint32, tp_status uint32) of the packets of one
    TPACKET_V3 block image, offsets relative to block_offset."""
    block = np.ascontiguousarray(block, np.uint8)
    o = np.empty(cap, np.uint64)
    ln = np.empty(cap, np.uint32)
    st = np.empty(cap, np.uint32)
    n = ctypes.c_uint64()
    check(lib.pnetgpu_tpacket3_walk(ctypes.c_void_p(block.ctypes.data), block.nbytes, block_offset,
                                    ctypes.c_void_p(o.ctypes.data), ctypes.c_void_p(ln.ctypes.data),
                                    ctypes.c_void_p(st.ctypes.data), cap, ctypes.byref(n)), "pnetgpu_tpacket3_walk")
    k = n.value
    return o[:k], ln[:k], st[:k]


class AfPacket:
    """A TPACKET_V3 receive ring on one interface (None = all). Needs CAP_NET_RAW:
    PermissionError otherwise."""

    def __init__(self, ifname=None, block_bytes=1 << 20, n_blocks=16, retire_ms=10):
        h = ctypes.c_void_p()
        rc = lib.pnetgpu_afp_open((ifname or "").encode(), block_bytes, n_blocks, retire_ms, ctypes.byref(h))
        if rc == ESYS:
            e = ctypes.get_errno()
            raise PermissionError(e, "AF_PACKET ring (needs CAP_NET_RAW)")
        check(rc, "pnetgpu_afp_open")
        self.h = h
        base, nbytes = ctypes.c_void_p(), ctypes.c_uint64()
        bb, nb = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib.pnetgpu_afp_ring(h, ctypes.byref(base), ctypes.byref(nbytes), ctypes.byref(bb), ctypes.byref(nb)),
              "pnetgpu_afp_ring")
        # the mapping as a numpy view: Ring.feed_region ships straight from it
        self.ring = np.ctypeslib.as_array(ctypes.cast(base, ctypes.POINTER(ctypes.c_uint8)), (nbytes.value,))
        self.block_bytes, self.n_blocks = bb.value, nb.value
        cap = bb.value // 32 + 1
        self._o = np.empty(cap, np.uint64)
        self._l = np.empty(cap, np.uint32)
        self._s = np.empty(cap, np.uint32)

    def next_block(self, timeout_ms=100):
        """(block, offsets, lengths, tp_status) of the next retired block (offsets
        into self.ring), or None on timeout. release(block) once consumed."""
        n, blk = ctypes.c_uint64(), ctypes.c_uint32()
        rc = lib.pnetgpu_afp_next_block(self.h, timeout_ms, ctypes.c_void_p(self._o.ctypes.data),
                                        ctypes.c_void_p(self._l.ctypes.data), ctypes.c_void_p(self._s.ctypes.data),
                                        len(self._o), ctypes.byref(n), ctypes.byref(blk))
        if rc == EEMPTY:
            return None
        check(rc, "pnetgpu_afp_next_block")
        k = n.value
        return blk.value, self._o[:k].copy(), self._l[:k].copy(), self._s[:k].copy()

    def release(self, block):
        check(lib.pnetgpu_afp_release_block(self.h, block), "pnetgpu_afp_release_block")

    def fanout(self, group_id, fanout_type="hash", defrag=False, rollover=False):
        """Join PACKET_FANOUT group group_id (pnet_datalink's FanoutOption)."""
        flags = (0x8000 if defrag else 0) | (0x1000 if rollover else 0)
        check(lib.pnetgpu_afp_fanout(self.h, group_id, FANOUT[fanout_type], flags), "pnetgpu_afp_fanout")

    def promiscuous(self, on=True):
        check(lib.pnetgpu_afp_promiscuous(self.h, 1 if on else 0), "pnetgpu_afp_promiscuous")

    def stats(self):
        p, d = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.pnetgpu_afp_stats(self.h, ctypes.byref(p), ctypes.byref(d)), "pnetgpu_afp_stats")
        return p.value, d.value

    def close(self):
        if self.h:
            self.ring = None
            lib.pnetgpu_afp_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


__all__ = ["AfPacket", "tpacket3_walk", "TP_STATUS_CSUMNOTREADY", "PnetGpuError"]
