"""examples/pcapdump.c: packetdump.rs over a pcap file with the per-packet work
on the GPU. CPU: the Rust-Display restatements the expected text relies on, and
that the binary is built. GPU: its stdout equals packetdump's lines (restated in
tests/packetdump_fmt.py from the oracle's records) for edge, random, ARP,
unknown-ethertype, ICMP echo and IPv6-address-format frames, with and without
the checksum suffix."""
import os
import subprocess

import numpy as np
import pytest

from tests import framegen
from tests.packetdump_fmt import line, v6
from tests.pcaputil import write_pcap, write_pcapng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "libpnet_amd", "build", "pcapdump")


def a6(*segs):
    return b"".join(s.to_bytes(2, "big") for s in segs)


@pytest.mark.parametrize("segs,text", [
    # Rust std Ipv6Addr Display examples (core::net docs and tests)
    ((0, 0, 0, 0, 0, 0, 0, 0), "::"),
    ((0, 0, 0, 0, 0, 0, 0, 1), "::1"),
    ((0, 0, 0, 0, 0, 0xffff, 0xc00a, 0x2ff), "::ffff:192.10.2.255"),
    ((0x2001, 0xdb8, 0, 0, 0, 0, 0, 1), "2001:db8::1"),
    ((1, 0, 0, 2, 0, 0, 0, 3), "1:0:0:2::3"),
    ((1, 0, 0, 2, 0, 0, 3, 4), "1::2:0:0:3:4"),
    ((1, 0, 2, 0, 3, 0, 4, 0), "1:0:2:0:3:0:4:0"),
    ((0, 0, 0, 0, 0, 0, 0xc00a, 0x2ff), "::c00a:2ff"),
    ((0xfe80, 0, 0, 0, 0, 0, 0, 0), "fe80::"),
])
def test_ipv6_display(segs, text):
    assert v6(a6(*segs)) == text


def test_pcapdump_built():
    assert os.access(EXE, os.X_OK), "run `make -C libpnet_amd` (build())"


def special_frames(rng):
    out = []
    # ARP request/reply (42 B and 60 B padded) and a truncated one
    for op, pad in ((1, 0), (2, 18)):
        f = bytearray(rng.integers(0, 256, 42 + pad, dtype=np.uint8).tobytes())
        f[12:14] = b"\x08\x06"
        f[14 + 6:14 + 8] = op.to_bytes(2, "big")
        out.append(bytes(f))
    f = bytearray(rng.integers(0, 256, 14 + 27, dtype=np.uint8).tobytes())
    f[12:14] = b"\x08\x06"
    out.append(bytes(f))
    # unknown ethertypes (LLDP, VLAN with flags 0, a random one)
    for et in (0x88CC, 0x8100, 0x1234):
        f = bytearray(rng.integers(0, 256, 60, dtype=np.uint8).tobytes())
        f[12:14] = et.to_bytes(2, "big")
        out.append(bytes(f))
    # ICMP echo request / reply / other types, over IPv4 and IPv6, short echoes
    for kind in ("icmp", "icmp_over6"):
        for t in (0, 8, 3, 11):
            for l4 in (4, 7, 8, 64):
                f = bytearray(framegen.build_frame(rng, kind, l4))
                f[-l4] = t
                out.append(bytes(f))
    # IPv6 address formats
    for src, dst in ((a6(0, 0, 0, 0, 0, 0, 0, 1), a6(0, 0, 0, 0, 0, 0xffff, 0x0a00, 0x0001)),
                     (a6(0x2001, 0xdb8, 0, 0, 1, 0, 0, 1), a6(0, 0, 0, 0, 0, 0, 0, 0)),
                     (a6(0xfe80, 0, 0, 0, 0x1234, 0, 0, 0), a6(1, 2, 3, 4, 5, 6, 7, 8))):
        for kind in ("udp6", "tcp6", "icmp6"):
            f = bytearray(framegen.build_frame(rng, kind, 40))
            f[22:38], f[38:54] = src, dst
            out.append(bytes(f))
    # unknown protocols (IPv4 GRE, IPv6 hop-by-hop with flags 0)
    f = bytearray(framegen.build_frame(rng, "udp", 30))
    f[23] = 47
    out.append(bytes(f))
    f = bytearray(framegen.build_frame(rng, "udp6", 30))
    f[20] = 0
    out.append(bytes(f))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("csum,fmt", [(False, "pcap"), (True, "pcap"), (True, "pcapng")])
def test_pcapdump_matches_packetdump_lines(tmp_path, csum, fmt):
    """pcapng captures (Enhanced / Simple / obsolete Packet Blocks over two
    interfaces and two sections) print the same lines as classic pcap ones."""
    rng = np.random.default_rng(77)
    frames = special_frames(rng) + framegen.edge_frames(rng) + framegen.random_frames(rng, 3000)
    p = tmp_path / f"dump.{fmt}"
    if fmt == "pcap":
        write_pcap(p, frames)
    else:
        write_pcapng(p, frames, kinds=(["epb", "pb", "epb", "spb"] * len(frames))[:len(frames)], n_if=2,
                     sections=2)
    args = [EXE, "-i", "eth7"] + (["-c"] if csum else []) + [str(p)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr
    got = r.stdout.splitlines()
    want = [line(f, "eth7", csum) for f in frames]
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"frame {i} ({len(frames[i])} B): got {g!r} want {w!r}"


@pytest.mark.gpu
def test_pcapdump_many_batches(tmp_path):
    """More records than one ring slot holds (2^18 frames): order and text kept
    across slots, waits and a partly filled last batch."""
    rng = np.random.default_rng(78)
    base = framegen.random_frames(rng, 500, max_len=200)
    frames = [base[i % len(base)] for i in range(300_001)]
    p = tmp_path / "big.pcap"
    write_pcap(p, frames)
    r = subprocess.run([EXE, str(p)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr
    want_base = [line(f) for f in base]
    got = r.stdout.splitlines()
    assert len(got) == len(frames)
    assert all(g == want_base[i % len(base)] for i, g in enumerate(got))


@pytest.mark.gpu
def test_pcapdump_empty_and_bad(tmp_path):
    p = tmp_path / "empty.pcap"
    write_pcap(p, [])
    r = subprocess.run([EXE, str(p)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout == ""
    q = tmp_path / "bad.pcap"
    q.write_bytes(b"not a pcap at all" * 4)
    r = subprocess.run([EXE, str(q)], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "pcapdump" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("linktype", [101, 229])
def test_pcapdump_raw_ip_capture(tmp_path, linktype):
    """A raw-IP capture (tun device) runs with PNETGPU_RX_L3: the same lines as
    the Ethernet capture of the same packets, plus the unknown-version line."""
    rng = np.random.default_rng(79)
    frames = special_frames(rng) + framegen.random_frames(rng, 2000)
    pkts = [f[14:] for f in frames if len(f) >= 14] + [b"", b"\x75" + bytes(30)]
    p = tmp_path / "raw.pcap"
    write_pcap(p, pkts, linktype=linktype)
    r = subprocess.run([EXE, "-c", str(p)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr
    got = r.stdout.splitlines()
    want = [line(f, "pcap", True, l3mode=True) for f in pkts]
    assert got == want
    assert got[-1] == "[pcap]: Unknown packet: IP version 7; length: 31"



def test_pcapdump_live_usage_and_bad_interface():
    """-l IFACE: argument errors exit 2; an unknown interface (or a denied
    packet socket) exits 1 with the reason, before any GPU call."""
    r = subprocess.run([EXE, "-l", "lo", "extra.pcap"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and "-l IFACE" in r.stderr
    r = subprocess.run([EXE, "-l", "no-such-if0", "-n", "1", "-w", "10"], capture_output=True, text=True,
                       timeout=30)
    assert r.returncode == 1
    assert "no-such-if0: invalid argument" in r.stderr or "not permitted" in r.stderr


def _live_in_netns(tmp_path):
    """pcapdump -l lo inside a private user + network namespace (where this
    process has no CAP_NET_RAW): tests/netns_loopback.py --pcapdump."""
    from tests.test_netns_loopback import run_in_netns
    out, _ = run_in_netns(["--pcapdump", os.path.join("libpnet_amd", "build", "pcapdump")], tmp_path)
    assert out["got"] == out["want"] and len(out["want"]) == 40, out


@pytest.mark.gpu
def test_pcapdump_live_loopback(tmp_path):
    """Live mode on `lo`: UDP datagrams sent while pcapdump -l captures come
    back as packetdump's UDP lines (ports and UDP length as sent). Where this
    process has no CAP_NET_RAW (the GPU box), the same run happens in a private
    network namespace (tests/netns_loopback.py); skips only where that is
    refused too."""
    import socket
    import time
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    port = rx.getsockname()[1]
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.bind(("127.0.0.1", 0))
    sport = tx.getsockname()[1]
    p = subprocess.Popen([EXE, "-l", "lo", "-w", "3000"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True)
    try:
        time.sleep(2.0)   # socket open + HIP context before the traffic starts
        if p.poll() is not None:
            err = p.stderr.read()
            if "not permitted" in err:
                rx.close()
                tx.close()
                return _live_in_netns(tmp_path)
            pytest.fail("pcapdump -l lo exited early: " + err)
        want = set()
        for i in range(40):
            tx.sendto(b"pnetgpu-live" + bytes(i), ("127.0.0.1", port))
            want.add("[lo]: UDP Packet: 127.0.0.1:%d > 127.0.0.1:%d; length: %d" % (sport, port, 8 + 12 + i))
        try:
            out, err = p.communicate(timeout=30)
        except subprocess.TimeoutExpired:   # other loopback traffic keeps it from going idle
            p.kill()
            out, err = p.communicate()
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
        rx.close()
        tx.close()
    assert p.returncode in (0, -9), err
    got = {ln for ln in out.splitlines() if ("127.0.0.1:%d" % port) in ln}
    if not got:
        pytest.skip("no loopback traffic visible to a packet socket here")
    assert got == want
