"""Loader for tests/golden/reference_kats.json (the reference's own KATs)."""
import json
import os

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_kats.json")


def load():
    with open(PATH) as fh:
        vecs = json.load(fh)["vectors"]
    for v in vecs:
        v["data"] = bytes.fromhex(v.get("data", ""))
    return vecs


def by_kind(*kinds):
    return [v for v in load() if v["kind"] in kinds]


def getter_frame(v):
    """An Ethernet frame whose receive dispatch reaches the view a "getters"
    vector describes, with that view's bytes (the reference test's) in place."""
    d = v["data"]
    view = v["view"]

    def ipv4(proto, l4):
        h = bytearray(20)
        h[0] = 0x45
        h[2:4] = (20 + len(l4)).to_bytes(2, "big")
        h[8], h[9] = 64, proto
        h[12:20] = bytes([192, 168, 0, 1, 192, 168, 0, 199])
        return bytes(h) + bytes(l4)

    if view == "ethernet":
        return d
    eth = bytes(12)
    if view == "ipv4":
        return eth + b"\x08\x00" + d
    if view == "ipv6":
        return eth + b"\x86\xdd" + d
    if view == "udp":
        return eth + b"\x08\x00" + ipv4(17, d)
    if view == "tcp":
        return eth + b"\x08\x00" + ipv4(6, d)
    if view == "icmpv6":
        h = bytearray(40)
        h[0] = 0x60
        h[4:6] = len(d).to_bytes(2, "big")
        h[6], h[7] = 58, 64
        h[23] = h[39] = 1
        return eth + b"\x86\xdd" + bytes(h) + d
    raise ValueError(view)
