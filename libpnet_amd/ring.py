"""Python binding of the host batch producer and pcap reader (include/pnetgpu_ring.h).

    ring = Ring(batch_bytes=64 << 20, batch_frames=1 << 18)
    for frame in pcap_frames("trace.pcap"):          # a DataLinkReceiver::next() stream
        for batch in ring.feed(frame):               # finished batches as they complete
            ...                                       # batch.records: host numpy columns
    for batch in ring.drain(): ...
"""
import ctypes

import numpy as np

from ._lib import DEFS, RxColumns, check, lib
from .engine import COLUMNS, COUNTER_NAMES, context

EFULL, EBUSY, EEMPTY = DEFS["PNETGPU_EFULL"], DEFS["PNETGPU_EBUSY"], DEFS["PNETGPU_EEMPTY"]


class RingBatch(ctypes.Structure):
    _fields_ = [("id", ctypes.c_uint64), ("n_frames", ctypes.c_uint64), ("frames", ctypes.c_void_p),
                ("offsets", ctypes.c_void_p), ("lengths", ctypes.c_void_p), ("cols", RxColumns)]


def _setup():
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.pnetgpu_ring_create.restype = i32
    lib.pnetgpu_ring_create.argtypes = [vp, u64, u32, u32, ctypes.POINTER(vp)]
    lib.pnetgpu_ring_destroy.restype = None
    lib.pnetgpu_ring_destroy.argtypes = [vp]
    lib.pnetgpu_ring_push.restype = i32
    lib.pnetgpu_ring_push.argtypes = [vp, vp, u32]
    lib.pnetgpu_ring_push_many.restype = i32
    lib.pnetgpu_ring_push_many.argtypes = [vp, vp, vp, vp, u64, ctypes.POINTER(u64)]
    lib.pnetgpu_ring_submit.restype = i32
    lib.pnetgpu_ring_submit.argtypes = [vp, ctypes.POINTER(u64)]
    lib.pnetgpu_ring_wait.restype = i32
    lib.pnetgpu_ring_wait.argtypes = [vp, ctypes.POINTER(RingBatch)]
    lib.pnetgpu_pcap_open.restype = i32
    lib.pnetgpu_pcap_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
    lib.pnetgpu_pcap_next.restype = i32
    lib.pnetgpu_pcap_next.argtypes = [vp, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(u32)]
    lib.pnetgpu_pcap_close.restype = None
    lib.pnetgpu_pcap_close.argtypes = [vp]


_setup()


class Batch:
    """A finished ring batch. With copy=False the arrays are views of the ring's
    pinned memory, valid until the ring's next wait (the C-ABI contract)."""

    def __init__(self, rb, copy=True):
        n = int(rb.n_frames)
        self.id, self.n = int(rb.id), n
        cp = (lambda a: a.copy()) if copy else (lambda a: a)
        self.offsets = cp(np.ctypeslib.as_array(ctypes.cast(rb.offsets, ctypes.POINTER(ctypes.c_uint64)), (n,)))
        self.lengths = cp(np.ctypeslib.as_array(ctypes.cast(rb.lengths, ctypes.POINTER(ctypes.c_uint32)), (n,)))
        nbytes = int(self.offsets[-1] + self.lengths[-1]) if n else 0
        self.frames = cp(np.ctypeslib.as_array(ctypes.cast(rb.frames, ctypes.POINTER(ctypes.c_uint8)),
                                               (max(nbytes, 1),))[:nbytes])
        self.records = {}
        for c, (_, npdt, shape) in COLUMNS.items():
            ptr = getattr(rb.cols, c)
            itemsize = np.dtype(npdt).itemsize
            ct = {1: ctypes.c_uint8, 2: ctypes.c_uint16, 4: ctypes.c_uint32}[itemsize]
            a = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), (n,) + shape) if n else np.zeros(
                (0,) + shape, npdt)
            self.records[c] = cp(a).view(npdt)
        ctr = np.ctypeslib.as_array(ctypes.cast(rb.cols.counters, ctypes.POINTER(ctypes.c_uint64)),
                                    (len(COUNTER_NAMES),))
        self.counters = dict(zip(COUNTER_NAMES, (int(x) for x in ctr)))


class Ring:
    """Pinned host batches -> asynchronous GPU verification (three rotating slots)."""

    def __init__(self, batch_bytes=64 << 20, batch_frames=1 << 18, device=0, copy=True, flags=0):
        self.ctx = context(device)
        self.copy = copy
        h = ctypes.c_void_p()
        check(lib.pnetgpu_ring_create(self.ctx.handle, batch_bytes, batch_frames, flags, ctypes.byref(h)),
              "pnetgpu_ring_create")
        self.h = h
        self.pending = 0

    def close(self):
        if getattr(self, "h", None):
            lib.pnetgpu_ring_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _wait(self):
        rb = RingBatch()
        rc = lib.pnetgpu_ring_wait(self.h, ctypes.byref(rb))
        if rc == EEMPTY:
            return None
        check(rc, "pnetgpu_ring_wait")
        self.pending -= 1
        return Batch(rb, self.copy)

    def submit(self):
        bid = ctypes.c_uint64()
        check(lib.pnetgpu_ring_submit(self.h, ctypes.byref(bid)), "pnetgpu_ring_submit")
        if bid.value != (1 << 64) - 1:
            self.pending += 1

    def feed(self, frame):
        """Push one frame; yields every batch that had to be completed to make room."""
        buf = (ctypes.c_uint8 * max(1, len(frame))).from_buffer_copy(bytes(frame) or b"\0")
        while True:
            rc = lib.pnetgpu_ring_push(self.h, buf, len(frame))
            if rc == 0:
                return
            if rc == EFULL:
                self.submit()
                continue
            if rc == EBUSY:
                b = self._wait()
                if b is not None:
                    yield b
                continue
            check(rc, "pnetgpu_ring_push")

    def feed_many(self, buf, offsets, lengths):
        """Push frames buf[offsets[i], +lengths[i]) (host arrays); yields completed batches."""
        buf = np.ascontiguousarray(buf, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        lengths = np.ascontiguousarray(lengths, np.uint32)
        i, n = 0, len(offsets)
        pushed = ctypes.c_uint64()
        while i < n:
            rc = lib.pnetgpu_ring_push_many(self.h, ctypes.c_void_p(buf.ctypes.data),
                                            ctypes.c_void_p(offsets[i:].ctypes.data),
                                            ctypes.c_void_p(lengths[i:].ctypes.data), n - i, ctypes.byref(pushed))
            if rc == 0:
                i += pushed.value
                if i < n:
                    self.submit()
                continue
            if rc == EFULL:
                self.submit()
                continue
            if rc == EBUSY:
                b = self._wait()
                if b is not None:
                    yield b
                continue
            check(rc, "pnetgpu_ring_push_many")

    def drain(self):
        """Submit the partial batch and yield every outstanding batch."""
        self.submit()
        while True:
            b = self._wait()
            if b is None:
                return
            yield b


def pcap_frames(path):
    """Frames of a classic Ethernet pcap file, as bytes (pcap.rs:92,168-179 receiver)."""
    h = ctypes.c_void_p()
    check(lib.pnetgpu_pcap_open(str(path).encode(), ctypes.byref(h)), "pnetgpu_pcap_open")
    try:
        fp = ctypes.POINTER(ctypes.c_uint8)()
        ln = ctypes.c_uint32()
        while True:
            rc = lib.pnetgpu_pcap_next(h, ctypes.byref(fp), ctypes.byref(ln))
            if rc == EEMPTY:
                return
            check(rc, "pnetgpu_pcap_next")
            yield ctypes.string_at(fp, ln.value)
    finally:
        lib.pnetgpu_pcap_close(h)
