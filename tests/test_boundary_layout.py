"""The boundary's struct layouts, three ways (CPU only): the C header as the
compiler lays it out, the ctypes mirror in libpnet_amd/_lib.py and ring.py, and
the Rust #[repr(C)] mirror in INTEGRATION.md §2 (the binding a pnet maintainer
would paste; pnet_macros_support/src/packet.rs:19-73 is the trait surface it
serves). A C file asserting every ctypes offset with _Static_assert must
compile, the Rust field lists must name the same fields in the same order with
types of the same size, and every entry point of the public headers must be
declared in the Rust extern block."""
import ctypes
import os
import re
import subprocess

import pytest

import libpnet_amd as lp
from libpnet_amd import _lib, ring

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRUCTS = {"pnetgpu_batch": _lib.Batch, "pnetgpu_rx_columns": _lib.RxColumns,
           "pnetgpu_ring_batch": ring.RingBatch, "pnetgpu_slice_desc": _lib.SliceDesc,
           "pnetgpu_ring_stats": ring.RingStats}
RUST_SIZES = {"u8": 1, "u16": 2, "u32": 4, "u64": 8, "c_int": 4, "f64": 8}


def test_ctypes_offsets_match_the_c_header(tmp_path):
    lines = ['#include <stddef.h>', '#include "pnetgpu.h"', '#include "pnetgpu_ring.h"']
    for cname, cls in STRUCTS.items():
        lines.append(f'_Static_assert(sizeof({cname}) == {ctypes.sizeof(cls)}, "sizeof {cname}");')
        for fname, _ in cls._fields_:
            off = getattr(cls, fname).offset
            lines.append(f'_Static_assert(offsetof({cname}, {fname}) == {off}, "{cname}.{fname}");')
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines) + "\n")
    p = subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def _rust_structs():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*pub struct (\w+) \{([^{}]*)\}", text):
        body = re.sub(r"//[^\n]*", "", m.group(2))
        out[m.group(1)] = re.findall(r"pub (\w+): ([^,\n]+)", body)
    return out


def _rust_layout(fields, structs):
    """repr(C) offsets of a Rust field list (pointers 8 B; nested structs by name)."""
    off, align_max, offs = 0, 1, []
    for name, ty in fields:
        ty = ty.strip()
        if ty.startswith("*"):
            size = align = 8
        elif ty in RUST_SIZES:
            size = align = RUST_SIZES[ty]
        else:
            size, align = _rust_layout(structs[ty], structs)[1:]
        off = (off + align - 1) // align * align
        offs.append((name, off))
        off += size
        align_max = max(align_max, align)
    return offs, (off + align_max - 1) // align_max * align_max, align_max


@pytest.mark.parametrize("cname", sorted(STRUCTS))
def test_rust_mirror_matches_the_c_header(cname):
    structs = _rust_structs()
    assert cname in structs, f"INTEGRATION.md has no #[repr(C)] {cname}"
    offs, size, _ = _rust_layout(structs[cname], structs)
    cls = STRUCTS[cname]
    assert [n for n, _ in offs] == [n for n, _ in cls._fields_]
    assert offs == [(n, getattr(cls, n).offset) for n, _ in cls._fields_]
    assert size == ctypes.sizeof(cls)


def test_rust_extern_block_declares_every_entry_point():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    declared = set(re.findall(r"pub fn (\w+)\(", text))
    for h in ("pnetgpu.h", "pnetgpu_ring.h", "pnetgpu_afpacket.h", "pnetgpu_util.h"):
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", h)).read(), flags=re.S)
        for fn in re.findall(r"^\s*(?:int|void|const char\*|uint\w+)\s+\**(pnetgpu_\w+)\s*\(", src, re.M):
            assert fn in declared, f"{h}: {fn} missing from the INTEGRATION.md Rust binding"
            assert hasattr(lp.lib, fn), fn


def test_rust_abi_version_constant():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    m = re.search(r"PNETGPU_ABI_VERSION: c_int = (\d+);", text)
    assert m and int(m.group(1)) == lp.DEFS["PNETGPU_ABI_VERSION"]
