"""CPU tests of the native pcap reader (pnetgpu_pcap_*): every byte order and
timestamp resolution, empty records, and rejection of non-Ethernet captures."""
import struct

import numpy as np
import pytest

import libpnet_amd as lp
from libpnet_amd._lib import PnetGpuError
from tests import framegen
from tests.pcaputil import write_pcap


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
