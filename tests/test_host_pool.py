"""The batch producer's host pass (pnetgpu_batch_pack = the pnetgpu_ring_push_many
pass, host_pool.cpp) on the CPU: bit-identical batches at every thread count,
the same cut as frame-by-frame pushes, and a persistent pool sized from the
affinity mask (no more workers than the CPUs the process may run on, none
created per call). The producer it replaces hands frames over one at a time
(pnet_datalink/src/linux.rs:362-403, lib.rs:227-230)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _frames(kind, n, seed=3, gaps=False):
    rng = np.random.default_rng(seed)
    if kind == "imix":
        lens = rng.choice(np.array([64, 576, 1500], np.uint32), size=n, p=[7 / 12, 4 / 12, 1 / 12]).astype(np.uint32)
    elif kind == "jumbo":
        lens = np.full(n, 9000, np.uint32)
    else:
        lens = np.full(n, 64, np.uint32)
    step = lens.astype(np.uint64) + (rng.integers(0, 3, n).astype(np.uint64) * 7 if gaps else 0)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(step[:-1], dtype=np.uint64)
    buf = rng.integers(0, 256, size=int(offs[-1] + lens[-1]), dtype=np.uint8)
    return buf, offs, lens


def _expect(buf, offs, lens, cap):
    """Frame-by-frame pushes: the longest prefix whose bytes fit cap."""
    k = int(np.searchsorted(np.cumsum(lens, dtype=np.uint64), np.uint64(cap), side="right"))
    packed = np.concatenate([buf[int(o):int(o) + int(ln)] for o, ln in zip(offs[:k], lens[:k])]) if k else \
        np.zeros(0, np.uint8)
    return k, packed


@pytest.mark.parametrize("kind,n,cap,gaps", [
    ("udp64", 1 << 17, 64 << 20, False),     # all fit, one run per chunk
    ("imix", 1 << 17, 4 << 20, False),       # cut inside the push, re-split evenly
    ("imix", 1 << 17, 1 << 30, True),        # non-adjacent frames: a copy per frame
    ("jumbo", 5000, 64 << 20, False),        # 9000-B frames: 7456 fit a 64-MiB batch
    ("imix", 1000, 1 << 20, True),           # below the parallel threshold: serial pass
])
def test_batch_pack_matches_single_pushes(kind, n, cap, gaps):
    import libpnet_amd as lp
    buf, offs, lens = _frames(kind, n, gaps=gaps)
    dst = np.zeros(cap, np.uint8) if cap <= (64 << 20) else np.zeros(int(lens.sum()) + 64, np.uint8)
    do = np.zeros(n, np.uint64)
    dl = np.zeros(n, np.uint32)
    k, b = lp.batch_pack(buf, offs, lens, dst, do, dl)
    ek, packed = _expect(buf, offs, lens, dst.size)
    assert k == ek and b == packed.size
    assert np.array_equal(dst[:b], packed)
    assert np.array_equal(dl[:k], lens[:k])
    want_off = np.zeros(k, np.uint64)
    want_off[1:] = np.cumsum(lens[:k - 1], dtype=np.uint64)
    assert np.array_equal(do[:k], want_off)


def test_batch_pack_first_frame_too_large():
    import libpnet_amd as lp
    buf, offs, lens = _frames("jumbo", 4)
    with pytest.raises(lp.PnetGpuError):
        lp.batch_pack(buf, offs, lens, np.zeros(8999, np.uint8), np.zeros(4, np.uint64), np.zeros(4, np.uint32))


_CHILD = r"""
import json, os, sys
import numpy as np
os.sched_setaffinity(0, {cpus})
sys.path.insert(0, {root!r})
import libpnet_amd as lp
from tests.test_host_pool import _frames, _expect
tasks = lambda: len(os.listdir("/proc/self/task"))
before = tasks()
threads = lp.host_threads()
buf, offs, lens = _frames("imix", 1 << 17, seed=5)
dst = np.zeros(8 << 20, np.uint8); do = np.zeros(1 << 17, np.uint64); dl = np.zeros(1 << 17, np.uint32)
k, b = lp.batch_pack(buf, offs, lens, dst, do, dl)
after1 = tasks()
for _ in range(5):
    lp.batch_pack(buf, offs, lens, dst, do, dl)
after2 = tasks()
ek, packed = _expect(buf, offs, lens, dst.size)
print(json.dumps({{"threads": threads, "new1": after1 - before, "new2": after2 - after1,
                   "ok": bool(k == ek and np.array_equal(dst[:b], packed))}}))
"""


def _child(cpus, env_extra=None):
    env = dict(os.environ)
    env.pop("PNETGPU_HOST_THREADS", None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, "-c", _CHILD.format(cpus=cpus, root=ROOT)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 2, reason="needs 2 CPUs")
def test_pool_sized_from_affinity_two_cpus():
    cpus = set(sorted(os.sched_getaffinity(0))[:2])
    r = _child(cpus)
    assert r["threads"] == 2
    assert r["new1"] <= 1          # the caller plus at most one worker
    assert r["new2"] == 0          # persistent: later passes start no thread
    assert r["ok"]


def test_pool_one_cpu_runs_serially():
    cpus = {sorted(os.sched_getaffinity(0))[0]}
    r = _child(cpus)
    assert r["threads"] == 1 and r["new1"] == 0 and r["new2"] == 0 and r["ok"]


def test_pool_env_override():
    cpus = set(sorted(os.sched_getaffinity(0))[:1])
    r = _child(cpus, {"PNETGPU_HOST_THREADS": "3"})
    assert r["threads"] == 3 and r["new1"] <= 2 and r["new2"] == 0 and r["ok"]


def test_ring_stats_and_pack_argument_checks():
    """The ring statistics entry points and the pack reject NULL handles and
    arrays before touching anything (no GPU involved)."""
    import ctypes
    import libpnet_amd as lp
    from libpnet_amd import ring
    st = ring.RingStats()
    einval = lp.DEFS["PNETGPU_EINVAL"]
    assert lp.lib.pnetgpu_ring_stats_get(None, ctypes.byref(st)) == einval
    assert lp.lib.pnetgpu_ring_stats_reset(None) == einval
    k, b = ctypes.c_uint64(), ctypes.c_uint64()
    assert lp.lib.pnetgpu_batch_pack(None, None, None, 4, None, 0, None, None, ctypes.byref(k), ctypes.byref(b)) \
        == einval
    assert lp.lib.pnetgpu_batch_pack(None, None, None, 0, None, 0, None, None, ctypes.byref(k), ctypes.byref(b)) == 0
    assert k.value == 0 and b.value == 0
    assert ctypes.sizeof(ring.RingStats) == 96       # 8 u64 + 3 f64 + 2 u32 (the C layout: test_boundary_layout)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="no toolchain")
def test_push_compact_descriptors_match_full_ones():
    """The ring push's compact (u32 / u16) descriptors — the ones it ships — equal
    its u64 / u32 ones for pushes starting at any slot fill level, serial and
    parallel, cut or whole (tools/pack_compact_check.cpp, CPU only)."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "libpnet_amd"), "compact-check"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert "pack_compact_check: ok" in r.stdout
