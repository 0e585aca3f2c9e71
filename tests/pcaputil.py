"""Minimal classic-pcap writer for tests (LINKTYPE_ETHERNET)."""
import struct


def write_pcap(path, frames, nanos=False, big_endian=False, snaplen=262144, linktype=1):
    e = ">" if big_endian else "<"
    magic = 0xA1B23C4D if nanos else 0xA1B2C3D4
    with open(path, "wb") as fh:
        fh.write(struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, snaplen, linktype))
        for i, f in enumerate(frames):
            fh.write(struct.pack(e + "IIII", 1700000000 + i, i, len(f), len(f)))
            fh.write(f)
