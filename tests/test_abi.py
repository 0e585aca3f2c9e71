"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
function the public headers declare, agrees with the oracle on the status/record
constants, and rejects bad arguments — without making any compute call."""
import ctypes
import os
import re
import subprocess

import pytest

import libpnet_amd as lp
from libpnet_amd import _lib
from oracle import coracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    headers = sorted(os.path.join(ROOT, "include", h) for h in os.listdir(os.path.join(ROOT, "include"))
                     if h.endswith(".h"))
    assert set(_lib.HEADERS) == set(headers), "libpnet_amd._lib.HEADERS must list every public header"
    for h in headers:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(pnetgpu_\w+)\s*\(", src))
    return sorted(names)


def test_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", lp.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (\w+)", out))
    decl = declared_functions()
    assert len(decl) >= 11
    missing = [d for d in decl if d not in exported]
    assert not missing, missing
    for d in decl:
        assert hasattr(lp.lib, d)


def test_abi_version_and_strerror():
    assert lp.lib.pnetgpu_abi_version() == lp.DEFS["PNETGPU_ABI_VERSION"] == 3
    for code in (0, -1, -2, -3, -4, -5, -6, -7, -8, -9, -99):
        assert lp.lib.pnetgpu_strerror(code)


def test_status_constants_match_oracle():
    hdr = open(os.path.join(ROOT, "oracle", "pnet_oracle.h")).read()
    for name, val in re.findall(r"#define (ORACLE_ST_\w+)\s+(0x[0-9a-fA-F]+)u", hdr):
        assert lp.DEFS["PNET_ST_" + name[len("ORACLE_ST_"):]] == int(val, 16), name


def test_column_dtypes_match_oracle_record():
    from libpnet_amd.engine import COLUMNS
    for c, (_, npdt, shape) in COLUMNS.items():
        f = coracle.REC_DTYPE.fields[c][0]
        assert f.base.itemsize == __import__("numpy").dtype(npdt).itemsize, c
        assert tuple(f.shape) == tuple(shape), c


def test_argument_validation_without_gpu():
    L = lp.lib
    assert L.pnetgpu_ctx_create(0, None) == lp.DEFS["PNETGPU_EINVAL"]
    assert L.pnetgpu_device_count(None) == lp.DEFS["PNETGPU_EINVAL"]
    assert L.pnetgpu_rx_process(None, None, None, None) == lp.DEFS["PNETGPU_EINVAL"]
    assert L.pnetgpu_checksum_slices(None, None, 0, 0, None, None, None, None, None) == lp.DEFS["PNETGPU_EINVAL"]
    h = ctypes.c_void_p()
    rc = L.pnetgpu_ctx_create(10 ** 6, ctypes.byref(h))
    assert rc == lp.DEFS["PNETGPU_ENODEV"] and not h.value
    L.pnetgpu_ctx_destroy(None)


def test_include_headers_compile_as_c():
    for h in ("pnetgpu.h", "pnetgpu_synth.h", "pnetgpu_ring.h", "pnetgpu_afpacket.h", "pnetgpu_util.h"):
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c",
                        os.path.join(ROOT, "include", h)], check=True)


def test_compact_slice_descriptor_packing():
    """slice_descriptors packs (offset, length, skipword) exactly as the C struct
    pnetgpu_slice_desc lays them out (u32, u16, u16 little-endian), and refuses
    values the compact form cannot hold."""
    import ctypes
    import numpy as np
    import pytest
    from libpnet_amd import _lib
    offs, lens, skips = [0, 5, 0xFFFFFFFF], [20, 0, 0xFFFF], [5, 0xFFFF, 0]
    t = lp.slice_descriptors(offs, lens, skips)
    raw = t.numpy().tobytes()
    arr = (_lib.SliceDesc * 3).from_buffer_copy(raw)
    assert ctypes.sizeof(_lib.SliceDesc) == 8
    assert [(d.offset, d.length, d.skipword) for d in arr] == list(zip(offs, lens, skips))
    with pytest.raises(ValueError):
        lp.slice_descriptors([1 << 32], [1], [0])
    with pytest.raises(ValueError):
        lp.slice_descriptors([0], [1 << 16], [0])
    assert np.asarray(lp.slice_descriptors([], [], [])).size == 0


def test_tuning_entry_points_without_gpu():
    """pnetgpu_ctx_set_tuning / get_tuning / sched_conflicts refuse a NULL
    context and unknown keys (no GPU needed); every PNETGPU_TUNE_* key has a
    Python name."""
    import ctypes

    from libpnet_amd import engine
    from libpnet_amd._lib import DEFS, lib
    assert lib.pnetgpu_ctx_set_tuning(None, 0, -1) == DEFS["PNETGPU_EINVAL"]
    v = ctypes.c_int64()
    assert lib.pnetgpu_ctx_get_tuning(None, 0, ctypes.byref(v)) == DEFS["PNETGPU_EINVAL"]
    c = ctypes.c_uint64()
    assert lib.pnetgpu_ctx_sched_conflicts(None, ctypes.byref(c)) == DEFS["PNETGPU_EINVAL"]
    keys = sorted(v for k, v in DEFS.items() if k.startswith("PNETGPU_TUNE_"))
    assert keys == list(range(DEFS["PNETGPU_NTUNE"]))
    assert sorted(engine.TUNING_KEYS.values()) == keys


def test_environment_read_only_at_context_creation():
    """The product path reads no environment variable per call: the only
    getenv calls in the C++ sources are tuning_from_env (called by
    pnetgpu_ctx_create) and the host pool's size (compute_threads, whose result
    host_threads() caches for the process)."""
    import re
    src_dir = os.path.join(ROOT, "libpnet_amd", "csrc")
    for f in sorted(os.listdir(src_dir)):
        text = open(os.path.join(src_dir, f)).read()
        hits = [m.start() for m in re.finditer(r"\bgetenv\s*\(", text)]
        if f == "host_pool.cpp":
            assert len(hits) == 1
            fn = text.rfind("\nunsigned compute_threads(", 0, hits[0])
            assert fn >= 0 and text.find("\n}\n", fn) > hits[0]
            assert text.count("g_threads = compute_threads()") == 2
            continue
        if f != "abi.cpp":
            assert not hits, f
            continue
        assert len(hits) == 1
        fn = text.rfind("\nvoid tuning_from_env(", 0, hits[0])
        assert fn >= 0 and text.find("\n}\n", fn) > hits[0]
        assert "tuning_from_env(c);" in text[text.index("int pnetgpu_ctx_create"):]


def test_desc_size_hint_rule():
    """pnetgpu_desc_size_hint: the tail shape a descriptor batch's host-side
    lengths call for (include/pnetgpu.h) — host arithmetic only."""
    import numpy as np
    import libpnet_amd as lp
    L, J = lp.DESC_HINT_LARGE, lp.DESC_HINT_JUMBO
    assert lp.desc_size_hint(np.zeros(0, np.uint32)) == 0
    assert lp.desc_size_hint(np.full(1000, 1500)) == L                      # MTU traffic
    assert lp.desc_size_hint(np.full(1000, 768)) == L
    assert lp.desc_size_hint(np.full(1000, 767)) == 0
    assert lp.desc_size_hint(np.full(1000, 9000)) == J                      # jumbo traffic
    assert lp.desc_size_hint(np.tile([64] * 7 + [9000], 100)) == J          # 95 % of the bytes jumbo
    imix = lp.synth.lengths("imix", 100000, seed=1)
    assert lp.desc_size_hint(imix) == 0                                     # IMIX: the mixed shape
    assert lp.desc_size_hint(np.array([64] * 1 + [1500] * 15)) == L         # 15/16 large
    assert lp.desc_size_hint(np.array([64] * 2 + [1500] * 15)) == 0
    mixed_jumbo = np.array([1500] * 10 + [9000])                            # 9000 of 24000 B: not jumbo
    assert lp.desc_size_hint(mixed_jumbo) == L
    assert _lib.lib.pnetgpu_desc_size_hint(None, 5) == 0
