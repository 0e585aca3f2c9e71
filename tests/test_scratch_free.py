"""No shipped kernel uses scratch (private segment) memory.

A select between a kernel argument and a loop-carried value, or a lane-variable
pick from a granule array, can make the compiler place registers in a stack
array: the slice kernels ran 10 % (12 B/lane) to 5x (96 B/lane) slower that
way (profiles/r03/slices/README.md, profiles/r04/slice_retest/README.md), and
nothing in the results shows it. This reads the gfx950 code object embedded in
the built libpnetgpu.so (clang offload bundle in .hip_fatbin) and checks every
kernel's AMDGPU metadata: private_segment_fixed_size 0 and no dynamic stack.
CPU only.
"""
import os
import struct

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "libpnet_amd", "libpnetgpu.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _gfx950_code_object(blob):
    at = blob.find(MAGIC)
    assert at >= 0, "no clang offload bundle in libpnetgpu.so"
    (n,) = struct.unpack_from("<Q", blob, at + len(MAGIC))
    p = at + len(MAGIC) + 8
    for _ in range(n):
        off, size, tlen = struct.unpack_from("<QQQ", blob, p)
        triple = blob[p + 24:p + 24 + tlen].decode()
        p += 24 + tlen
        if "amdgcn" in triple and "gfx950" in triple:
            return blob[at + off:at + off + size]
    raise AssertionError("no gfx950 code object in the bundle")


def _amdgpu_metadata(elf):
    assert elf[:4] == b"\x7fELF" and elf[4] == 2, "expected a 64-bit ELF code object"
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for k in range(shnum):
        sh = shoff + k * shentsize
        stype, = struct.unpack_from("<I", elf, sh + 4)
        if stype != 7:   # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        q, end = off, off + size
        while q < end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, q)
            name = elf[q + 12:q + 12 + namesz].rstrip(b"\0")
            d0 = q + 12 + ((namesz + 3) & ~3)
            if name == b"AMDGPU" and ntype == 32:   # NT_AMDGPU_METADATA (msgpack)
                return elf[d0:d0 + descsz]
            q = d0 + ((descsz + 3) & ~3)
    raise AssertionError("no NT_AMDGPU_METADATA note in the code object")


def test_no_kernel_uses_scratch():
    msgpack = pytest.importorskip("msgpack")
    if not os.path.exists(LIB):
        pytest.skip("libpnetgpu.so not built")
    with open(LIB, "rb") as fh:
        blob = fh.read()
    meta = msgpack.unpackb(_amdgpu_metadata(_gfx950_code_object(blob)), raw=False)
    kernels = meta["amdhsa.kernels"]
    assert len(kernels) >= 20, f"expected every receive/slice instantiation, found {len(kernels)}"
    bad = [(k[".name"], k[".private_segment_fixed_size"], k.get(".uses_dynamic_stack", False))
           for k in kernels if k[".private_segment_fixed_size"] or k.get(".uses_dynamic_stack", False)]
    assert not bad, f"kernels with scratch: {bad}"
