"""The plain-C example (examples/rx_verify.c) against the C-ABI: built by
libpnet_amd/Makefile with gcc, linked only to libpnetgpu.so and the HIP runtime.
CPU: the binary exists and resolves its libraries. GPU: it runs both the
device-resident and the zero-copy ring path and finds exactly the planted
corruptions (its exit status)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "libpnet_amd", "build", "rx_verify")


def test_example_built_and_linked():
    assert os.access(EXE, os.X_OK), "run `make -C libpnet_amd` (build())"
    out = subprocess.run(["ldd", EXE], capture_output=True, text=True, check=True).stdout
    assert "libpnetgpu.so" in out and "not found" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 1 << 20])
def test_example_runs(n):
    r = subprocess.run([EXE, str(n)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")
