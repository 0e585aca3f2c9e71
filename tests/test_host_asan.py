"""Host code under AddressSanitizer + UBSan (CPU only): the synthetic-frame
producer, the classic-pcap and pcapng readers (fuzzed) and the C-ABI argument validation, built from
sanitized objects into one executable (libpnet_amd/Makefile `asan-test`)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"), reason="no toolchain")
def test_host_code_asan_ubsan_clean():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "libpnet_amd"), "asan-test"], capture_output=True,
                       text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ok (0 failures)" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
