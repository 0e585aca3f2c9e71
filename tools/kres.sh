#!/bin/bash
# Per-kernel VGPR / spill / LDS / occupancy of rx_kernel.hip (extra args: -D defines)
cd "$(dirname "$0")/../libpnet_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../include -Icsrc --offload-arch=gfx950 "$@" -c csrc/rx_kernel.hip \
  -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for ln in sys.stdin:
    m = re.search(r"remark:\s+(.*?) \[-Rpass", ln)
    if not m: continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); print(); print(cur[:70], end="")
    elif any(t.startswith(k) for k in ("VGPRs:", "VGPRs Spill", "SGPRs Spill", "LDS Size", "Occupancy")):
        print("  " + t.replace(" [bytes/block]", ""), end="")
print()'
