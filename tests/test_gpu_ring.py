"""GPU end-to-end of the batch producer: frames pushed one by one (or from a pcap
replay) through the pinned ring come back with records identical to the oracle's."""
import ctypes
import re

import numpy as np
import pytest

import libpnet_amd as lp
from libpnet_amd._lib import PnetGpuError, check, lib
from oracle import coracle
from tests import framegen
from tests.pcaputil import write_pcap
from tests.test_gpu_parity import SHAPE_RE

pytestmark = pytest.mark.gpu


def check_batches(batches, frames, flags=0):
    got = sorted(batches, key=lambda b: b.id)
    assert [b.id for b in got] == list(range(len(got)))
    assert sum(b.n for b in got) == len(frames)
    i = 0
    for b in got:
        for k in range(b.n):
            assert bytes(b.frames[b.offsets[k]:b.offsets[k] + b.lengths[k]]) == frames[i + k]
        rec = coracle.rx_batch(b.frames, b.n, offsets=b.offsets, lengths=b.lengths, flags=flags)
        assert b.records, b.id
        for c, v in b.records.items():
            assert np.array_equal(v, rec[c]), (b.id, c)
        i += b.n


def test_ring_pcap_replay(tmp_path):
    rng = np.random.default_rng(9)
    frames = framegen.edge_frames(rng) + framegen.random_frames(rng, 4000, max_len=9000)
    p = tmp_path / "replay.pcap"
    write_pcap(p, frames)
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=700)     # many small batches: every slot state
    out = []
    for f in lp.pcap_frames(p):
        out.extend(ring.feed(f))
    out.extend(ring.drain())
    check_batches(out, frames)


def test_ring_feed_many_synth():
    w = lp.synth.make("imix", 50000, seed=6)
    frames = [bytes(w.buf[o:o + l]) for o, l in zip(w.offsets, w.lengths)]
    ring = lp.Ring(batch_bytes=4 << 20, batch_frames=1 << 14)
    out = list(ring.feed_many(w.buf, w.offsets, w.lengths)) + list(ring.drain())
    check_batches(out, frames)
    assert sum(b.counters["l4_csum_bad"] for b in out) == w.expect["l4_bad"]


@pytest.mark.parametrize("batch_bytes", [64 << 20, 8 << 20])
def test_ring_feed_many_large_pushes(batch_bytes):
    """Pushes of >= 2^16 frames split their descriptors and copies over host
    threads; with 8 MiB slots the byte capacity cuts each push (the serial
    path). Frames are spread with gaps, so copies break at chunk boundaries
    and inside chunks; batches equal the source frames and the oracle."""
    w = lp.synth.make("imix", 150000, seed=8)
    rng = np.random.default_rng(8)
    gaps = rng.integers(0, 3, w.offsets.size) * rng.integers(0, 40, w.offsets.size)
    offs = (w.offsets + np.cumsum(gaps)).astype(np.uint64)
    buf = np.zeros(int(offs[-1] + w.lengths[-1]) + 64, np.uint8)
    for o, no, n in zip(w.offsets.tolist(), offs.tolist(), w.lengths.tolist()):
        buf[no:no + n] = w.buf[o:o + n]
    ring = lp.Ring(batch_bytes=batch_bytes, batch_frames=1 << 18)
    out = sorted(list(ring.feed_many(buf, offs, w.lengths)) + list(ring.drain()), key=lambda b: b.id)
    assert [b.id for b in out] == list(range(len(out)))
    assert sum(b.n for b in out) == offs.size
    i = 0
    for b in out:
        assert np.array_equal(b.lengths, w.lengths[i:i + b.n])
        assert b.offsets[0] == 0 and np.array_equal(np.diff(b.offsets.astype(np.int64)), b.lengths[:-1])
        got = np.asarray(b.frames[:int(b.offsets[-1] + b.lengths[-1])])
        want = np.concatenate([buf[int(o):int(o) + int(l)] for o, l in zip(offs[i:i + b.n], w.lengths[i:i + b.n])])
        assert np.array_equal(got, want), b.id
        rec = coracle.rx_batch(b.frames, b.n, offsets=b.offsets, lengths=b.lengths)
        for c, v in b.records.items():
            assert np.array_equal(v, rec[c]), (b.id, c)
        i += b.n


@pytest.mark.parametrize("register", [False, True])
def test_ring_zero_copy_region(register):
    """submit_region ships frames straight from the caller's (pageable or
    registered) buffer; records equal the oracle's, frames are views of it."""
    w = lp.synth.make("imix", 60000, seed=8, corrupt_ppm=20000)
    frames = [bytes(w.buf[o:o + l]) for o, l in zip(w.offsets, w.lengths)]
    buf = np.array(w.buf, copy=True)
    ring = lp.Ring(batch_bytes=4 << 20, batch_frames=1 << 14, copy=True)
    reg = lp.HostRegistration(buf) if register else None
    try:
        out = list(ring.feed_region(buf, w.offsets, w.lengths)) + list(ring.drain())
    finally:
        if reg:
            reg.close()
    check_batches(out, frames)
    assert sum(b.counters["l4_csum_bad"] for b in out) == w.expect["l4_bad"]


def test_ring_zero_copy_pcap_image_after_pushes(tmp_path):
    """A pcap file image indexed by pnetgpu_pcap_scan and shipped zero-copy, after
    frames pushed one by one (submit_region first ships the filling batch)."""
    rng = np.random.default_rng(10)
    frames = framegen.edge_frames(rng) + framegen.random_frames(rng, 3000, max_len=9000)
    p = tmp_path / "replay.pcap"
    write_pcap(p, frames[1000:])
    img = np.fromfile(p, dtype=np.uint8)
    offs, lens = lp.pcap_index(img)
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=600)
    out = []
    for f in frames[:1000]:
        out.extend(ring.feed(f))
    out.extend(ring.feed_region(img, offs, lens))
    out.extend(ring.drain())
    check_batches(out, frames)


def test_ring_zero_copy_rejects_unsorted():
    buf = np.zeros(1 << 17, np.uint8)
    ring = lp.Ring(batch_bytes=1 << 16, batch_frames=64)
    with pytest.raises(PnetGpuError):                  # descending offsets
        list(ring.feed_region(buf, np.array([100, 50], np.uint64), np.array([60, 60], np.uint32)))
    with pytest.raises(ValueError):                     # a frame larger than batch_bytes
        list(ring.feed_region(buf, np.array([0], np.uint64), np.array([70000], np.uint32)))


def test_ring_column_subset():
    """Ring(columns=IPV4_COLUMNS): only those columns are computed and copied back."""
    w = lp.synth.make("udp64", 20000, seed=12, corrupt_ppm=20000)
    frames = [bytes(w.buf[i * 64:(i + 1) * 64]) for i in range(20000)]
    offs = np.arange(20000, dtype=np.uint64) * 64
    lens = np.full(20000, 64, np.uint32)
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=1 << 13, columns=lp.IPV4_COLUMNS)
    out = list(ring.feed_region(w.buf, offs, lens)) + list(ring.drain())
    assert all(set(b.records) == set(lp.IPV4_COLUMNS) for b in out)
    check_batches(out, frames)


def _oracle_check(b, ident):
    rec = coracle.rx_batch(np.asarray(b.frames), b.n, offsets=b.offsets, lengths=b.lengths)
    assert b.records, ident
    for c, v in b.records.items():
        assert np.array_equal(v, rec[c]), (ident, c)


@pytest.mark.parametrize("slots", [4, 6])
def test_ring_holds_a_batch_while_others_complete(slots):
    """With the consumer holding one batch (copy=False views of pinned memory),
    the other slots keep shipping: `slots - 2` more batches are submitted and
    finish on the GPU while it is held, the held batch's frames and records are
    untouched by them, and every batch equals the oracle."""
    import torch
    w = lp.synth.make("imix", 40000, seed=21, corrupt_ppm=20000)
    ring = lp.Ring(batch_bytes=2 << 20, batch_frames=4000, copy=False, slots=slots)
    assert ring.slots == slots
    per = 3000
    ranges = [(k * per, (k + 1) * per) for k in range(slots)]
    offs, lens = w.offsets, w.lengths

    def push(lo, hi):
        pushed = ctypes.c_uint64()
        check(lib.pnetgpu_ring_push_many(ring.h, ctypes.c_void_p(w.buf.ctypes.data),
                                       ctypes.c_void_p(offs[lo:].ctypes.data),
                                       ctypes.c_void_p(lens[lo:].ctypes.data), hi - lo,
                                       ctypes.byref(pushed)), "push_many")
        assert pushed.value == hi - lo
        ring.submit()

    push(*ranges[0])
    held = ring.wait()                      # batch 0 held from here on
    assert held.id == 0 and held.n == per
    snap = {c: v.copy() for c, v in held.records.items()}
    frames0 = np.asarray(held.frames).copy()
    for lo, hi in ranges[1:slots - 1]:      # every other slot but the filling one: in flight
        push(lo, hi)
    torch.cuda.synchronize()
    # the slots are all taken: one held, slots - 2 in flight, one filling
    for c, v in held.records.items():
        assert np.array_equal(v, snap[c]), c
    assert np.array_equal(np.asarray(held.frames), frames0)
    _oracle_check(held, 0)
    got = []
    while True:
        b = ring.wait()                     # releases the previous batch
        if b is None:
            break
        _oracle_check(b, b.id)
        got.append((b.id, b.n))
    assert got == [(k, per) for k in range(1, slots - 1)]
    ring.close()


def test_ring_slot_count_bounds():
    for bad in (0, 1, lp.DEFS["PNETGPU_RING_MAX_SLOTS"] + 1):
        with pytest.raises(PnetGpuError):
            lp.Ring(batch_bytes=1 << 16, batch_frames=64, slots=bad)
    r = lp.Ring(batch_bytes=1 << 16, batch_frames=64)
    assert r.slots == lp.DEFS["PNETGPU_RING_DEFAULT_SLOTS"] >= 4
    r.close()


@pytest.mark.parametrize("name,n,head", [("udp1500", 3000, "mtu"), ("imix", 20000, "mixed"), ("udp6_jumbo", 300, "jumbo")])
def test_ring_batches_carry_their_size_hint(name, n, head):
    """The ring counts each batch's large and jumbo frames as it fills it and
    ships the batch with its PNETGPU_DESC_HINT_*: MTU traffic runs the MTU
    shape, jumbo traffic the jumbo shape, IMIX the mixed one — records equal
    the oracle's either way."""
    w = lp.synth.make(name, n, seed=23, corrupt_ppm=20000)
    if w.stride:
        offs = np.arange(n, dtype=np.uint64) * np.uint64(w.stride)
        lens = np.full(n, w.frame_len, np.uint32)
    else:
        offs, lens = w.offsets, w.lengths
    frames = [bytes(w.buf[int(o):int(o) + int(l)]) for o, l in zip(offs, lens)]
    for region in (False, True):
        ring = lp.Ring(batch_bytes=16 << 20, batch_frames=1 << 15)
        out = list(ring.feed_region(w.buf, offs, lens) if region else ring.feed_many(w.buf, offs, lens))
        if not region:
            ring.submit()
        assert re.match(SHAPE_RE[head], lp.last_rx_kernel()), (region, lp.last_rx_kernel())
        out += list(ring.drain())
        ring.close()
        check_batches(out, frames)


@pytest.mark.parametrize("big", [False, True])
def test_ring_zero_copy_pcapng_image(tmp_path, big):
    """A pcapng capture (the other format libpcap's offline reader — and so
    pnet_datalink's pcap::from_file — takes), indexed in memory by
    pnetgpu_pcap_scan and shipped zero-copy: records equal the oracle's."""
    from tests.pcaputil import write_pcapng
    rng = np.random.default_rng(12)
    frames = framegen.edge_frames(rng) + framegen.random_frames(rng, 3000, max_len=9000)
    p = tmp_path / "replay.pcapng"
    write_pcapng(p, frames, big_endian=big, kinds=(["epb", "spb", "pb"] * len(frames))[:len(frames)], sections=3)
    img = np.fromfile(p, dtype=np.uint8)
    offs, lens = lp.pcap_index(img, batch=1000)
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=600)
    with lp.HostRegistration(img):
        out = list(ring.feed_region(img, offs, lens)) + list(ring.drain())
    check_batches(out, frames)
    assert list(lp.pcap_frames(p)) == frames


@pytest.mark.parametrize("producer", ["push_many", "zero_copy"])
def test_ring_jumbo_batches_and_stage_stats(producer):
    """configs[4]'s 9000-B IPv6/UDP frames through the bench's ring geometry
    (64-MiB slots: 7,456 jumbo frames a batch, past the reference producer's
    4096-B default read buffer, pnet_datalink/src/lib.rs:164-178): every batch
    equals the source frames and the oracle's records, the planted corruptions
    are all counted, and the ring's stage statistics account for every batch
    (PNETGPU_RING_STAGE_TIMES: H2D, kernel and D2H timed on the device)."""
    n = 20000
    w = lp.synth.make("udp6_jumbo", n, seed=12, corrupt_ppm=20000)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(w.stride)
    lens = np.full(n, w.frame_len, np.uint32)
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=True, stage_times=True)
    reg = lp.HostRegistration(w.buf) if producer == "zero_copy" else None
    try:
        feed = ring.feed_region if producer == "zero_copy" else ring.feed_many
        out = sorted(list(feed(w.buf, offs, lens)) + list(ring.drain()), key=lambda b: b.id)
        st = ring.stats()
        ring.reset_stats()
        z = ring.stats()
        assert z["host_threads"] == st["host_threads"] and z["batches"] == z["push_ns"] == 0 and z["h2d_ms"] == 0
    finally:
        ring.close()
        if reg:
            reg.close()
    assert [b.n for b in out] == [7456, 7456, n - 2 * 7456]
    i = 0
    for b in out:
        got = np.asarray(b.frames[:int(b.offsets[-1] + b.lengths[-1])])
        assert np.array_equal(got, w.buf[i * 9000:(i + b.n) * 9000]), b.id
        rec = coracle.rx_batch(b.frames, b.n, offsets=b.offsets, lengths=b.lengths)
        for c, v in b.records.items():
            assert np.array_equal(v, rec[c]), (b.id, c)
        i += b.n
    assert sum(b.counters["l4_csum_bad"] for b in out) == w.expect["l4_bad"] > 0
    assert sum(b.counters["bytes"] for b in out) == n * 9000
    assert st["batches"] == st["timed_batches"] == 3 and st["frames"] == n and st["bytes"] == n * 9000
    assert st["h2d_ms"] > 0 and st["kernel_ms"] > 0 and st["d2h_ms"] > 0
    assert st["wait_ns"] > 0 and st["submit_ns"] > 0 and st["host_threads"] >= 1
    assert st["push_ns"] > 0                       # push_many: copies + descriptors; zero-copy: descriptors


_AFFINITY_CHILD = r"""
import json, os, sys
os.sched_setaffinity(0, {cpus})
sys.path.insert(0, {root!r})
import numpy as np
import libpnet_amd as lp
from oracle import coracle
tasks = lambda: set(os.listdir("/proc/self/task"))
w = lp.synth.make("imix", 150000, seed=21)
ring = lp.Ring(batch_bytes=8 << 20, batch_frames=1 << 17, copy=True)
before = tasks()
out = sorted(list(ring.feed_many(w.buf, w.offsets, w.lengths)) + list(ring.drain()), key=lambda b: b.id)
st = ring.stats()
ring.close()
ok = sum(b.n for b in out) == 150000
i = 0
for b in out:
    rec = coracle.rx_batch(b.frames, b.n, offsets=b.offsets, lengths=b.lengths)
    ok = ok and all(np.array_equal(v, rec[c]) for c, v in b.records.items())
    ok = ok and np.array_equal(b.lengths, w.lengths[i:i + b.n])
    i += b.n
print(json.dumps({{"threads": lp.host_threads(), "stats_threads": st["host_threads"], "ok": bool(ok),
                   "batches": len(out), "push_ns": st["push_ns"]}}))
"""


def test_ring_push_many_two_cpus():
    """pnetgpu_ring_push_many in a process limited to two CPUs: its pool has
    two threads (the caller and one worker), every batch equals the oracle,
    and the ring's statistics report the pool size."""
    import json
    import os
    import subprocess
    import sys
    cpus = set(sorted(os.sched_getaffinity(0))[:2])
    if len(cpus) < 2:
        pytest.skip("needs 2 CPUs")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k != "PNETGPU_HOST_THREADS"}
    p = subprocess.run([sys.executable, "-c", _AFFINITY_CHILD.format(cpus=cpus, root=root)], cwd=root, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["threads"] == 2 and r["stats_threads"] == 2
    assert r["ok"] and r["batches"] > 3 and r["push_ns"] > 0


@pytest.mark.parametrize("batch_bytes", [64 << 20, 6 << 20])
def test_ring_zero_copy_large_regions(batch_bytes):
    """submit_region over pushes of >= 2^16 frames (the parallel descriptor pass:
    binary-searched cut, chunked order and fit checks): IMIX frames with gaps,
    cut by the slot's frame count (64 MiB) or its bytes (6 MiB); every batch
    equals the oracle and the frames are the caller's bytes."""
    w = lp.synth.make("imix", 200000, seed=23, corrupt_ppm=20000)
    rng = np.random.default_rng(23)
    gaps = rng.integers(0, 2, w.offsets.size) * rng.integers(0, 24, w.offsets.size)
    offs = (w.offsets + np.cumsum(gaps)).astype(np.uint64)
    buf = np.zeros(int(offs[-1] + w.lengths[-1]) + 64, np.uint8)
    for o, no, n in zip(w.offsets.tolist(), offs.tolist(), w.lengths.tolist()):
        buf[no:no + n] = w.buf[o:o + n]
    ring = lp.Ring(batch_bytes=batch_bytes, batch_frames=1 << 17, copy=True)
    out = sorted(list(ring.feed_region(buf, offs, w.lengths)) + list(ring.drain()), key=lambda b: b.id)
    ring.close()
    assert sum(b.n for b in out) == offs.size and len(out) >= 2
    i = 0
    for b in out:
        assert np.array_equal(b.lengths, w.lengths[i:i + b.n])
        assert np.array_equal(b.offsets.astype(np.uint64) + offs[i], offs[i:i + b.n])
        rec = coracle.rx_batch(b.frames, b.n, offsets=b.offsets, lengths=b.lengths)
        for c, v in b.records.items():
            assert np.array_equal(v, rec[c]), (b.id, c)
        i += b.n
    assert sum(b.counters["l4_csum_bad"] for b in out) == w.expect["l4_bad"]


def test_ring_zero_copy_large_region_overlap_rejected():
    """An overlap deep inside a push of 2^17 frames (inside the first batch,
    then past it) is rejected exactly where the serial contract rejects it:
    PNETGPU_EINVAL for the batch that contains it, the batches before it shipped."""
    n = 1 << 17
    lens = np.full(n, 64, np.uint32)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(64)
    buf = np.zeros(n * 64 + 64, np.uint8)
    for at in (5000, 100000):
        bad = offs.copy()
        bad[at] = bad[at - 1] + np.uint64(10)               # overlaps the frame before it
        ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 16, copy=True)
        got = []
        with pytest.raises(PnetGpuError):
            for b in ring.feed_region(buf, bad, lens):
                got.append(b.n)
        # the batches of frames before the overlap that completed before the error
        assert sum(got) <= (at // (1 << 16)) * (1 << 16)
        ring.close()


def _uniform_case(case, n=3000):
    """(frames, buffer, offsets, lengths, flags, whether any batch should ship
    fixed-stride) for one batch shape."""
    rng = np.random.default_rng(17)

    def synth(name, m, cut=None):
        w = lp.synth.make(name, m, seed=5)
        assert w.stride
        ln = cut or w.frame_len
        return [bytes(w.buf[i * w.stride:i * w.stride + ln]) for i in range(m)]
    gap, flags = 0, 0
    if case == "64_packed":
        fr, strided = synth("udp64", n), True
    elif case == "64_at_128":                  # TPACKET-like fixed frame slots
        fr, gap, strided = synth("udp64", n), 64, True
    elif case == "60_packed":                  # stride not a 16-B multiple: descriptors
        fr, strided = synth("udp64", n, cut=60), False
    elif case == "200_packed":                 # between the small and MTU kernels: descriptors
        fr, strided = synth("udp1500", n, cut=200), False
    elif case == "1500_packed":
        fr, strided = synth("udp1500", n), True
    elif case == "9000_packed":
        fr, strided = synth("udp6_jumbo", 400), True
    elif case == "64_vlan_flag":               # parse extensions: not the small kernel, descriptors
        fr, flags, strided = synth("udp64", n), lp.engine.RX_VLAN, False
    elif case == "64_ragged_gaps":             # uniform lengths, irregular spacing: descriptors
        fr, gap, strided = synth("udp64", n), None, False
    else:                                      # one frame a byte short: its batch keeps descriptors
        fr, strided = synth("udp64", n), None
        fr[n // 2] = fr[n // 2][:-1]
    lens = np.array([len(f) for f in fr], np.uint32)
    step = lens.astype(np.uint64) + (rng.integers(0, 4, len(fr)).astype(np.uint64) * 16 if gap is None
                                     else np.uint64(gap))
    offs = np.zeros(len(fr), np.uint64)
    offs[1:] = np.cumsum(step[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    for f, o in zip(fr, offs):
        buf[int(o):int(o) + len(f)] = np.frombuffer(f, np.uint8)
    return fr, buf, offs, lens, flags, strided


def _ships_strided(b, flags):
    """The ring's rule (ring.cpp ship_slot), restated from the waited batch."""
    off = np.asarray(b.offsets[:b.n], np.uint64)
    ln = np.asarray(b.lengths[:b.n], np.uint32)
    if b.n < 2 or ln.min() != ln.max():
        return False
    stride = int(off[1] - off[0])
    if not np.array_equal(off - off[0], np.arange(b.n, dtype=np.uint64) * np.uint64(stride)):
        return False
    L = int(ln[0])
    return (L <= 64 and stride % 16 == 0 and flags == 0) or L >= 768


@pytest.mark.parametrize("producer", ["push_many", "region"])
@pytest.mark.parametrize("case", ["64_packed", "64_at_128", "60_packed", "200_packed", "1500_packed", "9000_packed",
                                  "64_vlan_flag", "64_ragged_gaps", "one_short"])
def test_ring_uniform_batches_ship_fixed_stride(case, producer):
    """Batches of uniform frames at a constant stride ship as fixed-stride
    batches (no descriptors on the link) where the fixed-stride kernel is the
    one the size hint would reach; every other batch keeps its descriptors. The
    records equal the oracle's either way. The copying ring packs frames back to
    back, so its stride is the frame length whatever the source spacing."""
    fr, buf, offs, lens, flags, strided = _uniform_case(case)
    if producer == "push_many" and case in ("64_at_128", "64_ragged_gaps"):
        strided = True                          # packed back to back: stride 64
    ring = lp.Ring(batch_bytes=1 << 20, batch_frames=1024, flags=flags)
    try:
        feed = ring.feed_many if producer == "push_many" else ring.feed_region
        out = []
        for b in feed(buf, offs, lens):
            out.append((b, _ships_strided(b, flags)))
        for b in ring.drain():
            out.append((b, _ships_strided(b, flags)))
        check_batches([b for b, _ in out], fr, flags=flags)
        st = ring.stats()
    finally:
        ring.close()
    assert st["batches"] == len(out) >= 2
    n_strided = sum(s for _, s in out)
    assert st["stride_batches"] == n_strided
    assert st["desc_bytes"] == 6 * sum(b.n for b, s in out if not s)
    if strided is None:
        assert 0 < n_strided < len(out)
    else:
        assert (n_strided == len(out)) if strided else n_strided == 0


def _push_all(ring, buf, offs, lens):
    pushed = ctypes.c_uint64()
    check(lib.pnetgpu_ring_push_many(ring.h, ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                     ctypes.c_void_p(lens.ctypes.data), len(offs), ctypes.byref(pushed)),
          "pnetgpu_ring_push_many")
    assert pushed.value == len(offs)


@pytest.mark.parametrize("case", ["uniform_then_mixed", "single_frame", "uniform_then_single_push",
                                  "uniform_then_other_push", "mtu_then_small_frame"])
def test_ring_push_backfills_compact_descriptors(case):
    """While every frame of a slot has one length that ships fixed-stride, the
    pushes leave the compact descriptors out; a later push or single-frame push
    that breaks the pattern, or a batch that ships with descriptors after all
    (one frame), backfills them first. Every batch equals the oracle's."""
    fr, buf, offs, lens, _, _ = _uniform_case("1500_packed" if case == "mtu_then_small_frame" else "64_packed", 600)
    ring = lp.Ring(batch_bytes=4 << 20, batch_frames=4096)
    frames = []
    try:
        if case == "single_frame":
            _push_all(ring, buf, offs[:1], lens[:1])
            frames = fr[:1]
            want_stride = 0
        else:
            _push_all(ring, buf, offs[:500], lens[:500])
            frames = fr[:500]
            extra = {"uniform_then_mixed": [fr[500][:60], fr[501], fr[502][:33]],
                     "uniform_then_single_push": [fr[500]],
                     "uniform_then_other_push": [fr[500][:48]] * 3,
                     "mtu_then_small_frame": [fr[500][:100]]}[case]
            if case in ("uniform_then_single_push", "mtu_then_small_frame"):
                for f in extra:
                    list(ring.feed(f))
            else:
                eb = np.concatenate([np.frombuffer(f, np.uint8) for f in extra])
                el = np.array([len(f) for f in extra], np.uint32)
                eo = np.zeros(len(extra), np.uint64)
                eo[1:] = np.cumsum(el[:-1], dtype=np.uint64)
                _push_all(ring, eb, eo, el)
            frames = frames + extra
            want_stride = 1 if case == "uniform_then_single_push" else 0
        out = list(ring.drain())
        st = ring.stats()
    finally:
        ring.close()
    assert len(out) == 1
    check_batches(out, frames)
    assert st["stride_batches"] == want_stride
    assert st["desc_bytes"] == (0 if want_stride else 6 * len(frames))


@pytest.mark.parametrize("producer", ["push_many", "region"])
def test_ring_full_slot_stride_batch_at_bench_geometry(producer):
    """The bench's ring geometry with 64-B frames: 2^20 frames fill a 64-MiB
    slot exactly, so the fixed-stride batch's last frame ends at the slot's
    byte capacity (the small kernel reads to the granule tail and no further);
    both batches (full, then 1,000 frames) equal the oracle's records, and
    both shipped without descriptors."""
    from tests.test_gpu_parity import NTHREADS
    n = (1 << 20) + 1000
    w = lp.synth.make("udp64", n, seed=23, corrupt_ppm=5000)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(64)
    lens = np.full(n, 64, np.uint32)
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=True)
    try:
        feed = ring.feed_many if producer == "push_many" else ring.feed_region
        out = sorted(list(feed(w.buf, offs, lens)) + list(ring.drain()), key=lambda b: b.id)
        st = ring.stats()
    finally:
        ring.close()
    assert [b.n for b in out] == [1 << 20, 1000]
    assert st["stride_batches"] == 2 and st["desc_bytes"] == 0
    i = 0
    for b in out:
        rec = coracle.rx_batch(w.buf[i * 64:(i + b.n) * 64], b.n, stride=64, frame_len=64, nthreads=NTHREADS)
        for c, v in b.records.items():
            assert np.array_equal(v, rec[c]), (b.id, c)
        i += b.n
    assert sum(b.counters["l4_csum_bad"] for b in out) == w.expect["l4_bad"] > 0


def test_ring_alternating_pushes_describe_each_frame_once():
    """Uniform frames arriving through push_many and single pushes in turn keep
    the slot lazily described (no compact descriptors written, no repeated
    backfill); one odd frame at the end fills them in once for the whole slot
    and the batch ships with descriptors equal to the oracle's records."""
    fr, buf, offs, lens, _, _ = _uniform_case("64_packed", 3000)
    ring = lp.Ring(batch_bytes=4 << 20, batch_frames=4096)
    frames = []
    try:
        i = 0
        while i < 2900:
            _push_all(ring, buf, offs[i:i + 90], lens[i:i + 90])
            frames += fr[i:i + 90]
            list(ring.feed(fr[i + 90]))
            frames.append(fr[i + 90])
            i += 100
        st0 = ring.stats()
        list(ring.feed(fr[2999][:40]))
        frames.append(fr[2999][:40])
        out = list(ring.drain())
        st = ring.stats()
    finally:
        ring.close()
    assert st0["batches"] == 0 and len(out) == 1
    check_batches(out, frames)
    assert st["stride_batches"] == 0 and st["desc_bytes"] == 6 * len(frames)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_ring_random_push_sequences(seed):
    """A random sequence of single pushes, push_many runs (uniform or mixed
    lengths, 64-B or 1500-B or odd sizes) and early submits through a small
    ring: every batch equals its frames and the oracle's records, whichever way
    each batch shipped (fixed-stride or descriptors) and however its compact
    descriptors were written (during the push, skipped, or filled in later)."""
    rng = np.random.default_rng(seed)
    pool = {64: _uniform_case("64_packed", 400)[0], 1500: _uniform_case("1500_packed", 400)[0]}
    ring = lp.Ring(batch_bytes=256 << 10, batch_frames=700, copy=True)
    frames, out = [], []
    try:
        for _ in range(120):
            op = rng.integers(0, 4)
            size = int(rng.choice([64, 64, 1500]))
            src = pool[size]
            if op == 0:                                       # one frame, sometimes cut short
                f = src[int(rng.integers(0, len(src)))]
                if rng.random() < 0.2:
                    f = f[:int(rng.integers(14, len(f)))]
                out += list(ring.feed(f))
                frames.append(f)
            elif op in (1, 2):                                # a run through push_many
                k = int(rng.integers(1, 120))
                run = [src[int(j)] for j in rng.integers(0, len(src), k)]
                if op == 2 and k > 2:                         # mixed: one frame of another length
                    j = int(rng.integers(0, k))
                    run[j] = run[j][:int(rng.integers(14, len(run[j])))]
                b = np.concatenate([np.frombuffer(f, np.uint8) for f in run])
                ln = np.array([len(f) for f in run], np.uint32)
                of = np.zeros(k, np.uint64)
                of[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
                out += list(ring.feed_many(b, of, ln))
                frames += run
            else:                                             # ship what is there now
                ring.submit()
        out += list(ring.drain())
        st = ring.stats()
    finally:
        ring.close()
    check_batches(out, frames)
    assert st["batches"] == len(out) and st["frames"] == len(frames)
    assert 0 < st["stride_batches"] < len(out)
