"""Python binding of the host batch producer and pcap reader (include/pnetgpu_ring.h).

    ring = Ring(batch_bytes=64 << 20, batch_frames=1 << 18)
    for frame in pcap_frames("trace.pcap"):          # a DataLinkReceiver::next() stream
        for batch in ring.feed(frame):               # finished batches as they complete
            ...                                       # batch.records: host numpy columns
    for batch in ring.drain(): ...
"""
import ctypes

import numpy as np

from ._lib import ALL_COLUMN_NAMES, DEFS, RxColumns, check, lib
from .engine import COLUMNS, COUNTER_NAMES, context

EFULL, EBUSY, EEMPTY = DEFS["PNETGPU_EFULL"], DEFS["PNETGPU_EBUSY"], DEFS["PNETGPU_EEMPTY"]


STAGE_TIMES = DEFS["PNETGPU_RING_STAGE_TIMES"]


class RingBatch(ctypes.Structure):
    _fields_ = [("id", ctypes.c_uint64), ("n_frames", ctypes.c_uint64), ("frames", ctypes.c_void_p),
                ("offsets", ctypes.c_void_p), ("lengths", ctypes.c_void_p), ("cols", RxColumns)]


class RingStats(ctypes.Structure):
    """pnetgpu_ring_stats (include/pnetgpu_ring.h)."""
    _fields_ = [("batches", ctypes.c_uint64), ("frames", ctypes.c_uint64), ("bytes", ctypes.c_uint64),
                ("push_ns", ctypes.c_uint64), ("submit_ns", ctypes.c_uint64), ("wait_ns", ctypes.c_uint64),
                ("timed_batches", ctypes.c_uint64), ("desc_bytes", ctypes.c_uint64), ("h2d_ms", ctypes.c_double),
                ("kernel_ms", ctypes.c_double), ("d2h_ms", ctypes.c_double), ("host_threads", ctypes.c_uint32),
                ("stride_batches", ctypes.c_uint32)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


def _setup():
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.pnetgpu_ring_create.restype = i32
    lib.pnetgpu_ring_create.argtypes = [vp, u64, u32, u32, ctypes.POINTER(vp)]
    lib.pnetgpu_ring_create_ex.restype = i32
    lib.pnetgpu_ring_create_ex.argtypes = [vp, u64, u32, u32, u32, ctypes.POINTER(vp)]
    lib.pnetgpu_ring_slots.restype = u32
    lib.pnetgpu_ring_slots.argtypes = [vp]
    lib.pnetgpu_ring_release.restype = i32
    lib.pnetgpu_ring_release.argtypes = [vp]
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
    lib.pnetgpu_ring_set_columns.restype = i32
    lib.pnetgpu_ring_set_columns.argtypes = [vp, u64]
    lib.pnetgpu_ring_submit_region.restype = i32
    lib.pnetgpu_ring_submit_region.argtypes = [vp, vp, vp, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.pnetgpu_host_register.restype = i32
    lib.pnetgpu_host_register.argtypes = [vp, u64]
    lib.pnetgpu_host_unregister.restype = i32
    lib.pnetgpu_host_unregister.argtypes = [vp]
    lib.pnetgpu_pcap_scan.restype = i32
    lib.pnetgpu_pcap_scan.argtypes = [vp, u64, ctypes.POINTER(u64), vp, vp, u64, ctypes.POINTER(u64)]
    lib.pnetgpu_pcap_info.restype = i32
    lib.pnetgpu_pcap_info.argtypes = [vp, u64, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    lib.pnetgpu_ring_stats_get.restype = i32
    lib.pnetgpu_ring_stats_get.argtypes = [vp, ctypes.POINTER(RingStats)]
    lib.pnetgpu_ring_stats_reset.restype = i32
    lib.pnetgpu_ring_stats_reset.argtypes = [vp]
    lib.pnetgpu_host_threads.restype = u32
    lib.pnetgpu_host_threads.argtypes = []
    lib.pnetgpu_batch_pack.restype = i32
    lib.pnetgpu_batch_pack.argtypes = [vp, vp, vp, u64, vp, u64, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]


_setup()


class _Mem:
    """A raw memory range as a numpy array without building a ctypes array type
    per call (np.ctypeslib.as_array does, which cost ~1 ms per waited batch
    over its 20 arrays: a quarter of the ring's link rate at 78 GB/s)."""

    __slots__ = ("__array_interface__",)

    def __init__(self, ptr, shape, dtype):
        self.__array_interface__ = {"data": (ptr, False), "shape": shape, "typestr": np.dtype(dtype).str,
                                    "version": 3}


def _view(ptr, shape, dtype):
    if not ptr or not int(np.prod(shape)):
        return np.zeros(shape, dtype)
    return np.asarray(_Mem(ptr, shape, dtype))


class Batch:
    """A finished ring batch. With copy=False the arrays are views of the ring's
    pinned memory, valid until the ring's next wait or release (the C-ABI
    contract): the generators below release a batch when they resume after
    yielding it, so views must not outlive the consumer's loop iteration.
    The views are made on first use (offsets, lengths, frames, records): a
    consumer that reads only the counters costs one small view per batch, which
    keeps the ring at the link's rate (tools/probes/ring_probe.py)."""

    def __init__(self, rb, copy=True):
        n = int(rb.n_frames)
        self.id, self.n = int(rb.id), n
        self._ptr = (rb.offsets, rb.lengths, rb.frames)
        self._cols = {c: getattr(rb.cols, c) for c in COLUMNS}
        self._cache = {}
        ctr = _view(rb.cols.counters, (len(COUNTER_NAMES),), np.uint64)
        self.counters = dict(zip(COUNTER_NAMES, (int(x) for x in ctr)))
        if copy:                            # owned arrays, valid after the ring moves on
            self._cache = {"offsets": self.offsets.copy(), "lengths": self.lengths.copy()}
            self._cache["frames"] = self.frames.copy()
            self._cache["records"] = {c: v.copy() for c, v in self.records.items()}

    @property
    def offsets(self):
        if "offsets" not in self._cache:
            self._cache["offsets"] = _view(self._ptr[0], (self.n,), np.uint64)
        return self._cache["offsets"]

    @property
    def lengths(self):
        if "lengths" not in self._cache:
            self._cache["lengths"] = _view(self._ptr[1], (self.n,), np.uint32)
        return self._cache["lengths"]

    @property
    def frames(self):
        if "frames" not in self._cache:
            nbytes = int(self.offsets[-1] + self.lengths[-1]) if self.n else 0
            self._cache["frames"] = _view(self._ptr[2], (nbytes,), np.uint8)
        return self._cache["frames"]

    @property
    def records(self):
        """Host record columns by name (only the ones the ring computed)."""
        if "records" not in self._cache:
            self._cache["records"] = {c: _view(ptr, (self.n,) + COLUMNS[c][2], COLUMNS[c][1])
                                      for c, ptr in self._cols.items() if ptr}
        return self._cache["records"]


def host_threads():
    """Threads the producers' parallel passes use, the caller included (pnetgpu_host_threads)."""
    return int(lib.pnetgpu_host_threads())


def batch_pack(buf, offsets, lengths, dst, dst_offsets, dst_lengths, check_bounds=True):
    """pnetgpu_batch_pack: frames buf[offsets[i], +lengths[i]) back to back into dst
    (host arrays, no GPU), descriptors into dst_offsets / dst_lengths; returns
    (frames packed, bytes packed). Raises on PNETGPU_EFULL (first frame > dst).
    check_bounds=False skips the O(n) numpy check that every frame lies inside
    buf (for callers whose descriptors come from a scan of buf itself)."""
    buf = np.ascontiguousarray(buf, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    lengths = np.ascontiguousarray(lengths, np.uint32)
    n = len(offsets)
    for a, dt in ((dst, np.uint8), (dst_offsets, np.uint64), (dst_lengths, np.uint32)):
        if a.dtype != dt or not a.flags.c_contiguous:
            raise TypeError("dst arrays must be contiguous uint8 / uint64 / uint32")
    if len(lengths) != n or len(dst_offsets) < n or len(dst_lengths) < n:
        raise ValueError("offsets, lengths and the descriptor outputs must cover n frames")
    if check_bounds and n and int((offsets + lengths).max()) > buf.size:
        raise ValueError("a frame extends past buf")
    k, b = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib.pnetgpu_batch_pack(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(offsets.ctypes.data),
                                 ctypes.c_void_p(lengths.ctypes.data), n, ctypes.c_void_p(dst.ctypes.data), dst.size,
                                 ctypes.c_void_p(dst_offsets.ctypes.data), ctypes.c_void_p(dst_lengths.ctypes.data),
                                 ctypes.byref(k), ctypes.byref(b)), "pnetgpu_batch_pack")
    return int(k.value), int(b.value)


class Ring:
    """Pinned host batches -> asynchronous GPU verification (rotating slots: one
    filling, one held by the consumer, the rest in flight)."""

    def __init__(self, batch_bytes=64 << 20, batch_frames=1 << 18, device=0, copy=True, flags=0, columns=None,
                 slots=None, stage_times=False):
        """columns: names of the record columns to compute and copy back (default all);
        slots: slot count (default PNETGPU_RING_DEFAULT_SLOTS); stage_times: time each
        batch's H2D / kernel / D2H on the GPU (PNETGPU_RING_STAGE_TIMES, see stats())."""
        flags |= STAGE_TIMES if stage_times else 0
        self.ctx = context(device)
        self.copy = copy
        h = ctypes.c_void_p()
        slots = DEFS["PNETGPU_RING_DEFAULT_SLOTS"] if slots is None else slots
        check(lib.pnetgpu_ring_create_ex(self.ctx.handle, batch_bytes, batch_frames, flags, slots, ctypes.byref(h)),
              "pnetgpu_ring_create_ex")
        self.h = h
        self.slots = int(lib.pnetgpu_ring_slots(h))
        self.pending = 0
        if columns is not None:
            mask = 0
            for c in columns:
                mask |= 1 << ALL_COLUMN_NAMES.index(c)
            check(lib.pnetgpu_ring_set_columns(self.h, mask), "pnetgpu_ring_set_columns")

    def close(self):
        if getattr(self, "h", None):
            lib.pnetgpu_ring_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        """pnetgpu_ring_stats as a dict: host seconds inside push_many / submit /
        wait, device stage sums (stage_times rings), batches, frames, bytes."""
        st = RingStats()
        check(lib.pnetgpu_ring_stats_get(self.h, ctypes.byref(st)), "pnetgpu_ring_stats_get")
        return st.as_dict()

    def reset_stats(self):
        check(lib.pnetgpu_ring_stats_reset(self.h), "pnetgpu_ring_stats_reset")

    def _wait(self):
        rb = RingBatch()
        rc = lib.pnetgpu_ring_wait(self.h, ctypes.byref(rb))
        if rc == EEMPTY:
            return None
        check(rc, "pnetgpu_ring_wait")
        self.pending -= 1
        return Batch(rb, self.copy)

    def release(self):
        """Release the batch the last wait returned (pnetgpu_ring_release)."""
        check(lib.pnetgpu_ring_release(self.h), "pnetgpu_ring_release")

    def wait(self):
        """The oldest submitted batch (blocking), or None when nothing is in flight.
        It stays held (copy=False views valid) until the next wait or release."""
        return self._wait()

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
                    self.release()             # the consumer is done with it: refill its slot now
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
                    self.release()             # the consumer is done with it: refill its slot now
                continue
            check(rc, "pnetgpu_ring_push_many")

    def feed_region(self, buf, offsets, lengths):
        """Zero-copy: ship frames buf[offsets[i], +lengths[i]) (ascending, non-overlapping)
        straight from buf, one H2D per batch (pnetgpu_ring_submit_region); yields
        completed batches, whose `frames` view buf. Keep buf unchanged until they
        are consumed; register it (HostRegistration) for a direct DMA."""
        buf = np.ascontiguousarray(buf, np.uint8)
        offsets = np.ascontiguousarray(offsets, np.uint64)
        lengths = np.ascontiguousarray(lengths, np.uint32)
        i, n = 0, len(offsets)
        taken, bid = ctypes.c_uint64(), ctypes.c_uint64()
        while i < n:
            rc = lib.pnetgpu_ring_submit_region(self.h, ctypes.c_void_p(buf.ctypes.data),
                                                ctypes.c_void_p(offsets[i:].ctypes.data),
                                                ctypes.c_void_p(lengths[i:].ctypes.data), n - i, ctypes.byref(taken),
                                                ctypes.byref(bid))
            if rc == 0:
                i += taken.value
                self.pending += 1
                continue
            if rc == EBUSY:
                b = self._wait()
                if b is not None:
                    yield b
                    self.release()             # the consumer is done with it: refill its slot now
                continue
            if rc == EFULL:                      # frames pushed earlier are still filling: ship them
                before = self.pending
                self.submit()
                if self.pending == before:
                    raise ValueError(f"frame {i} ({int(lengths[i])} B) exceeds the ring's batch_bytes")
                continue
            check(rc, "pnetgpu_ring_submit_region")

    def drain(self):
        """Submit the partial batch and yield every outstanding batch."""
        self.submit()
        while True:
            b = self._wait()
            if b is None:
                return
            yield b
            self.release()


class HostRegistration:
    """Page-locks a host numpy array for direct DMA (pnetgpu_host_register) for
    the lifetime of the context."""

    def __init__(self, arr):
        self.arr = arr
        self.ptr = ctypes.c_void_p(arr.ctypes.data)
        check(lib.pnetgpu_host_register(self.ptr, arr.nbytes), "pnetgpu_host_register")

    def close(self):
        if self.ptr is not None:
            check(lib.pnetgpu_host_unregister(self.ptr), "pnetgpu_host_unregister")
            self.ptr = None

    def __enter__(self):
        return self.arr

    def __exit__(self, *exc):
        self.close()


def pcap_index(img, batch=1 << 16):
    """Record descriptors of an in-memory pcap or pcapng image (e.g. np.fromfile or
    np.memmap of the file): (offsets uint64, lengths uint32) of every record's
    captured bytes within img, for Ring.feed_region (pnetgpu_pcap_scan)."""
    img = np.ascontiguousarray(img, np.uint8)
    pos, n = ctypes.c_uint64(0), ctypes.c_uint64()
    offs, lens = [], []
    while True:
        o = np.empty(batch, np.uint64)
        ln = np.empty(batch, np.uint32)
        check(lib.pnetgpu_pcap_scan(ctypes.c_void_p(img.ctypes.data), img.nbytes, ctypes.byref(pos),
                                    ctypes.c_void_p(o.ctypes.data), ctypes.c_void_p(ln.ctypes.data), batch,
                                    ctypes.byref(n)), "pnetgpu_pcap_scan")
        offs.append(o[:n.value])
        lens.append(ln[:n.value])
        if pos.value >= img.nbytes or n.value == 0:
            break
    return np.concatenate(offs), np.concatenate(lens)


def pcap_info(img):
    """(link type, receive flags) of an in-memory pcap image: Ethernet (1) -> 0,
    raw IP (101 / 228 / 229) -> RX_L3 (pnetgpu_pcap_info)."""
    img = np.ascontiguousarray(img, np.uint8)
    lt, fl = ctypes.c_uint32(), ctypes.c_uint32()
    check(lib.pnetgpu_pcap_info(ctypes.c_void_p(img.ctypes.data), img.nbytes, ctypes.byref(lt), ctypes.byref(fl)),
          "pnetgpu_pcap_info")
    return lt.value, fl.value


def pcap_frames(path):
    """Frames of an Ethernet pcap or pcapng file, as bytes (pcap.rs:92,168-179 receiver)."""
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
