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


def _pad4(b):
    return b + bytes((-len(b)) % 4)


def _block(e, btype, body):
    body = _pad4(body)
    n = 12 + len(body)
    return struct.pack(e + "II", btype, n) + body + struct.pack(e + "I", n)


def pcapng_bytes(frames, big_endian=False, linktype=1, snaplen=0, kinds=None, n_if=1, sections=1, extras=True):
    """A pcapng image (the block format libpcap's offline reader, and so
    pnet_datalink's pcap::from_file, accepts): `sections` sections, each with a
    Section Header Block (with an option), `n_if` Interface Description Blocks
    of `linktype` / `snaplen`, and the frames spread over them as Enhanced
    Packet Blocks ("epb", round-robin over the interfaces, with options),
    Simple Packet Blocks ("spb", interface 0; captured = min(original, snaplen))
    or obsolete Packet Blocks ("pb") per `kinds` (a list as long as frames, or
    None = all EPB); with `extras`, a Name Resolution Block, an Interface
    Statistics Block and a custom block the reader must skip."""
    e = ">" if big_endian else "<"
    kinds = kinds or ["epb"] * len(frames)
    out = b""
    per = -(-len(frames) // sections) if frames else 0
    for s in range(sections):
        opt = struct.pack(e + "HH", 4, 5) + _pad4(b"tests") + struct.pack(e + "HH", 0, 0)   # shb_userappl
        out += _block(e, 0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1) + opt)
        for _ in range(n_if):
            out += _block(e, 1, struct.pack(e + "HHI", linktype, 0, snaplen))
        if extras:
            out += _block(e, 4, struct.pack(e + "HH", 0, 0))                      # NRB: end of records
            out += _block(e, 0x40000BAD, b"custom!")                               # custom block
        for i in range(s * per, min(len(frames), (s + 1) * per)):
            f, k = frames[i], kinds[i]
            if k == "epb":
                opt = struct.pack(e + "HH", 1, 3) + _pad4(b"hi!") + struct.pack(e + "HH", 0, 0)
                out += _block(e, 6, struct.pack(e + "IIIII", i % n_if, 0, i, len(f), len(f) + 7) + _pad4(f) + opt)
            elif k == "spb":
                out += _block(e, 3, struct.pack(e + "I", len(f)) + f)
            else:
                out += _block(e, 2, struct.pack(e + "HHIIII", i % n_if, 0, 0, i, len(f), len(f)) + f)
        if extras:
            out += _block(e, 5, struct.pack(e + "III", 0, 0, 0))                  # ISB
    return out


def write_pcapng(path, frames, **kw):
    with open(path, "wb") as fh:
        fh.write(pcapng_bytes(frames, **kw))
