#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch figures from a gfx950 assembly file
(`hipcc --save-temps` output): python tools/kstats.py file.s"""
import re
import sys

src = open(sys.argv[1]).read()
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", src, re.S):
    body = m.group(2)

    def g(k):
        x = re.search(r"\.amdhsa_" + k + r" (\d+)", body)
        return int(x.group(1)) if x else -1
    name = m.group(1)
    dem = re.sub(r"_ZN7pnetgpu12_GLOBAL__N_1", "", name)[:70]
    print(f"{dem:72s} vgpr={g('next_free_vgpr'):4d} agpr_off={g('accum_offset'):4d} sgpr={g('next_free_sgpr'):4d} "
          f"lds={g('group_segment_fixed_size'):6d} scratch={g('private_segment_fixed_size'):5d}")
