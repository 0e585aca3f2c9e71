"""The batch producer's host pool under ThreadSanitizer (CPU only): parallel
packs on the persistent pool while another thread packs concurrently, built
with -fsanitize=thread (libpnet_amd/Makefile `tsan-test`,
tools/host_tsan_test.cpp): no data race, every batch byte-identical."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"), reason="no toolchain")
def test_host_pool_tsan_clean():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "libpnet_amd"), "tsan-test"], capture_output=True,
                       text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ok (0 bad" in out
    assert "WARNING: ThreadSanitizer" not in out
