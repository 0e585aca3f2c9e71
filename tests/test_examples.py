"""The plain-C example (examples/rx_verify.c) against the C-ABI: built by
libpnet_amd/Makefile with gcc, linked only to libpnetgpu.so and the HIP runtime.
CPU: the binary exists and resolves its libraries. GPU: it runs the
device-resident path, the zero-copy ring path (6 slots, batches released as
read) and a 1500-B descriptor batch with its size hint, and finds exactly the
planted corruptions every way (its exit status)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "libpnet_amd", "build", "rx_verify")
SENDER = os.path.join(ROOT, "libpnet_amd", "build", "rs_sender")
UTIL = os.path.join(ROOT, "libpnet_amd", "build", "util_checksum")


def test_example_built_and_linked():
    for exe in (EXE, SENDER, UTIL):
        assert os.access(exe, os.X_OK), "run `make -C libpnet_amd` (build())"
        out = subprocess.run(["ldd", exe], capture_output=True, text=True, check=True).stdout
        assert "libpnetgpu.so" in out and "not found" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 1 << 20])
def test_example_runs(n):
    r = subprocess.run([EXE, str(n)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")


@pytest.mark.gpu
def test_rs_sender_fills_what_the_oracle_computes(tmp_path):
    """examples/rs_sender.c: rs_sender.rs's frame batch with zero checksum fields,
    filled on the GPU and written to a pcap; every written frame equals the
    oracle's fill of the same frame, and frame 0 carries 0xB8CA / 0xB94C."""
    import numpy as np
    import libpnet_amd as lp
    from oracle import coracle
    p = tmp_path / "tx.pcap"
    n = 50000
    r = subprocess.run([SENDER, str(n), str(p)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0xB8CA" in r.stdout and "0xB94C" in r.stdout
    frames = list(lp.pcap_frames(p))
    assert len(frames) == n and all(len(f) == 64 for f in frames)
    buf = np.frombuffer(b"".join(frames), np.uint8).copy()
    zeroed = buf.copy().reshape(n, 64)
    zeroed[:, 24:26] = 0
    zeroed[:, 40:42] = 0
    want, _ = coracle.tx_fill(np.concatenate([zeroed.reshape(-1), np.zeros(64, np.uint8)]), n, stride=64,
                              frame_len=64)
    assert np.array_equal(buf, want[: n * 64])



@pytest.mark.gpu
def test_util_checksum_example_reference_kats():
    """examples/util_checksum.c (pnetgpu_util.h from plain C, host bytes in,
    the word out) on the reference's own KATs: icmp.rs:82-108's checksums,
    udp.rs:58-100 (0x9178) and tcp.rs:288-357."""
    from tests import kats

    def run(*args):
        r = subprocess.run([UTIL, *args], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        return int(r.stdout.strip(), 16)

    for v in kats.by_kind("checksum"):
        assert run(bytes(v["data"]).hex(), str(v["skipword"])) == v["expected"], v["name"]
    v4 = {v["name"]: v for v in kats.by_kind("ipv4_checksum")}
    assert run("-4", bytes(v4["udp_ipv4_checksum"]["data"]).hex(), "3", "c0a80001", "c0a800c7", "17") == 0x9178
    assert run("-4", bytes(v4["tcp_ipv4_checksum"]["data"]).hex(), "8", "c0a80201", "c0a86f33", "6") == \
        v4["tcp_ipv4_checksum"]["expected"]
