"""CPU tests of the native pcap reader (pnetgpu_pcap_*): every byte order and
timestamp resolution, empty records, and rejection of non-Ethernet captures."""
import struct

import numpy as np
import pytest

import libpnet_amd as lp
from libpnet_amd._lib import PnetGpuError
from tests import framegen
from tests.pcaputil import pcapng_bytes, write_pcap, write_pcapng


@pytest.mark.parametrize("nanos", [False, True])
@pytest.mark.parametrize("big", [False, True])
def test_pcap_roundtrip(tmp_path, nanos, big):
    frames = framegen.random_frames(np.random.default_rng(4), 300) + [b""]
    p = tmp_path / "t.pcap"
    write_pcap(p, frames, nanos=nanos, big_endian=big)
    assert list(lp.pcap_frames(p)) == frames


def test_pcap_rejects_non_ethernet(tmp_path):
    p = tmp_path / "x.pcap"
    p.write_bytes(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 101))
    with pytest.raises(PnetGpuError):
        list(lp.pcap_frames(p))
    q = tmp_path / "y.pcap"
    q.write_bytes(b"not a pcap at all" * 4)
    with pytest.raises(PnetGpuError):
        list(lp.pcap_frames(q))


@pytest.mark.parametrize("nanos", [False, True])
@pytest.mark.parametrize("big", [False, True])
def test_pcap_index_matches_reader(tmp_path, nanos, big):
    """pnetgpu_pcap_scan over the file image finds the same records as the streaming
    reader, in several resumed calls (batch smaller than the record count)."""
    frames = framegen.random_frames(np.random.default_rng(5), 500) + [b""]
    p = tmp_path / "t.pcap"
    write_pcap(p, frames, nanos=nanos, big_endian=big)
    img = np.fromfile(p, dtype=np.uint8)
    offs, lens = lp.pcap_index(img, batch=64)
    assert len(offs) == len(frames)
    assert [bytes(img[o:o + n]) for o, n in zip(offs, lens)] == frames


def test_pcap_index_rejects_truncated_and_non_ethernet(tmp_path):
    p = tmp_path / "t.pcap"
    write_pcap(p, [b"\x01" * 100, b"\x02" * 60])
    img = np.fromfile(p, dtype=np.uint8)
    with pytest.raises(PnetGpuError):
        lp.pcap_index(img[:-10])                        # last record cut short
    bad = img.copy()
    bad[20] = 113                                       # LINKTYPE_LINUX_SLL: not supported
    with pytest.raises(PnetGpuError):
        lp.pcap_index(bad)
    with pytest.raises(PnetGpuError):
        lp.pcap_info(bad)


@pytest.mark.parametrize("linktype,flags", [(1, 0), (101, 4), (228, 4), (229, 4)])
def test_pcap_info_link_types(tmp_path, linktype, flags):
    """Ethernet captures need no flags; raw-IP ones (LINKTYPE_RAW / IPV4 / IPV6)
    need PNETGPU_RX_L3, and index like any other."""
    frames = [f[14:] for f in framegen.random_frames(np.random.default_rng(6), 50)] if flags else \
        framegen.random_frames(np.random.default_rng(6), 50)
    p = tmp_path / "t.pcap"
    write_pcap(p, frames, linktype=linktype)
    img = np.fromfile(p, dtype=np.uint8)
    assert lp.pcap_info(img) == (linktype, flags)
    assert flags == 0 or flags == lp.engine.RX_L3
    offs, lens = lp.pcap_index(img)
    assert [bytes(img[o:o + n]) for o, n in zip(offs, lens)] == frames


# ---- pcapng (libpcap's other offline format, pcap.rs:92 from_file) ---------

@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("kinds", ["epb", "spb", "pb", "mixed"])
def test_pcapng_roundtrip(tmp_path, big, kinds):
    """Streaming reader and in-memory indexer over pcapng: every byte order,
    Enhanced / Simple / obsolete Packet Blocks, several interfaces and sections,
    options and skipped block types; the frames come back as written."""
    frames = framegen.random_frames(np.random.default_rng(7), 400) + [b""]
    k = (["epb", "spb", "pb"] * len(frames))[:len(frames)] if kinds == "mixed" else [kinds] * len(frames)
    n_if = 1 if kinds in ("spb", "mixed") else 3
    p = tmp_path / "t.pcapng"
    write_pcapng(p, frames, big_endian=big, kinds=k, n_if=n_if, sections=1 if kinds == "spb" else 3)
    assert list(lp.pcap_frames(p)) == frames
    img = np.fromfile(p, dtype=np.uint8)
    offs, lens = lp.pcap_index(img, batch=37)                 # many resumed calls
    assert [bytes(img[o:o + n]) for o, n in zip(offs, lens)] == frames
    assert lp.pcap_info(img) == (1, 0)


def test_pcapng_simple_packet_blocks_honour_the_snap_length(tmp_path):
    """An SPB carries no captured length: it is min(original length, the
    interface's snap length) (the data past it is padding)."""
    frames = [bytes(range(256)) * 2, b"\x07" * 90]
    img = np.frombuffer(pcapng_bytes(frames, kinds=["spb", "spb"], snaplen=100), np.uint8)
    offs, lens = lp.pcap_index(img)
    assert list(lens) == [100, 90]
    assert bytes(img[offs[0]:offs[0] + 100]) == frames[0][:100]


def test_pcapng_raw_ip_link_type(tmp_path):
    frames = [f[14:] for f in framegen.random_frames(np.random.default_rng(8), 40)]
    img = np.frombuffer(pcapng_bytes(frames, linktype=101, n_if=2), np.uint8)
    assert lp.pcap_info(img) == (101, lp.engine.RX_L3)
    offs, lens = lp.pcap_index(img)
    assert [bytes(img[o:o + n]) for o, n in zip(offs, lens)] == frames
    p = tmp_path / "raw.pcapng"
    p.write_bytes(img.tobytes())
    with pytest.raises(PnetGpuError):                         # the streaming reader is Ethernet-only
        list(lp.pcap_frames(p))


def test_pcapng_rejects_malformed(tmp_path):
    frames = [b"\x01" * 100, b"\x02" * 61]
    good = pcapng_bytes(frames)
    img = np.frombuffer(good, np.uint8)
    for bad in (img[:-6],                                     # last block cut short
                np.concatenate([img, np.zeros(8, np.uint8)])):   # trailing garbage shorter than a block
        with pytest.raises(PnetGpuError):
            lp.pcap_index(bad)
    b = bytearray(good)
    b[len(b) - 4] ^= 1                                        # trailing length != leading length
    with pytest.raises(PnetGpuError):
        lp.pcap_index(np.frombuffer(bytes(b), np.uint8))
    b = bytearray(good)
    struct.pack_into("<I", b, 8, 0x11223344)                  # bad byte-order magic
    with pytest.raises(PnetGpuError):
        lp.pcap_index(np.frombuffer(bytes(b), np.uint8))
    # interfaces of different link types (libpcap refuses them too)
    two = pcapng_bytes(frames, n_if=1) + pcapng_bytes(frames, linktype=101, n_if=1)
    with pytest.raises(PnetGpuError):
        lp.pcap_index(np.frombuffer(two, np.uint8))
    # an EPB naming an interface that was never described
    lonely = pcapng_bytes(frames, n_if=1)
    epb_if = lonely.find(struct.pack("<II", 6, 12 + 20 + 100)) + 8
    b = bytearray(lonely)
    struct.pack_into("<I", b, epb_if, 5)
    with pytest.raises(PnetGpuError):
        lp.pcap_index(np.frombuffer(bytes(b), np.uint8))
    for path, data in (("a.pcapng", two), ("b.pcapng", bytes(b))):
        q = tmp_path / path
        q.write_bytes(data)
        with pytest.raises(PnetGpuError):
            list(lp.pcap_frames(q))


def _scan(img, pos, cap):
    import ctypes
    from libpnet_amd._lib import check, lib
    p, n = ctypes.c_uint64(pos), ctypes.c_uint64()
    o, ln = np.empty(cap, np.uint64), np.empty(cap, np.uint32)
    check(lib.pnetgpu_pcap_scan(ctypes.c_void_p(img.ctypes.data), img.nbytes, ctypes.byref(p),
                                ctypes.c_void_p(o.ctypes.data), ctypes.c_void_p(ln.ctypes.data), cap,
                                ctypes.byref(n)), "pnetgpu_pcap_scan")
    return p.value, list(zip(o[:n.value].tolist(), ln[:n.value].tolist()))


def test_pcapng_scan_resumes_and_restarts():
    """A pcapng scan in batches resumes where the thread's previous call of the
    same image stopped (no re-walk from byte 0); scans of two images interleaved,
    and a scan restarted at an earlier block boundary, still see each position's
    own section state (byte order, interfaces)."""
    rng = np.random.default_rng(8)
    fa = framegen.random_frames(rng, 120)
    fb = framegen.random_frames(rng, 90)
    a = np.frombuffer(pcapng_bytes(fa, big_endian=True, n_if=2, sections=3), np.uint8).copy()
    b = np.frombuffer(pcapng_bytes(fb, big_endian=False, n_if=3, sections=2), np.uint8).copy()
    want_a = list(zip(*[x.tolist() for x in lp.pcap_index(a, batch=1000)]))
    want_b = list(zip(*[x.tolist() for x in lp.pcap_index(b, batch=1000)]))
    got_a, got_b, pa, pb, stops = [], [], 0, 0, []
    while pa < a.nbytes or pb < b.nbytes:
        if pa < a.nbytes:
            stops.append(pa)
            pa, r = _scan(a, pa, 7)
            got_a += r
        if pb < b.nbytes:
            pb, r = _scan(b, pb, 5)
            got_b += r
    assert got_a == want_a and got_b == want_b
    # restarts at earlier stops of image a (not where the last call ended)
    for s in stops[::-1][:6]:
        _, r = _scan(a, s, 10 ** 6)
        assert r == [x for x in want_a if x[0] >= s]


def test_pcapng_scan_resume_checks_the_image_not_only_its_address():
    """A batched pcapng scan resumes with the section state its previous call
    stopped with only when the image is the same one: a different image of the
    same size rewritten into the same buffer (as allocator reuse would place
    it) is walked from its own headers again, so its records come out right."""
    import ctypes
    from libpnet_amd._lib import lib
    from tests.pcaputil import pcapng_bytes
    rng = np.random.default_rng(4)
    lens = rng.integers(60, 200, 40)
    fa = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in lens]
    fb = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in lens]
    a, b = pcapng_bytes(fa), pcapng_bytes(fb, big_endian=True)
    assert len(a) == len(b)
    buf = np.frombuffer(a, np.uint8).copy()
    offs = np.zeros(64, np.uint64)
    lns = np.zeros(64, np.uint32)
    pos, n = ctypes.c_uint64(0), ctypes.c_uint64()

    def scan(cap):
        rc = lib.pnetgpu_pcap_scan(ctypes.c_void_p(buf.ctypes.data), buf.size, ctypes.byref(pos),
                                   ctypes.c_void_p(offs.ctypes.data), ctypes.c_void_p(lns.ctypes.data), cap,
                                   ctypes.byref(n))
        assert rc == 0
        return [bytes(buf[int(o):int(o) + int(ln)]) for o, ln in zip(offs[:n.value], lns[:n.value])]

    assert scan(5) == fa[:5]
    buf[:] = np.frombuffer(b, np.uint8)        # another image, same size, same address
    assert scan(64) == fb[5:]
