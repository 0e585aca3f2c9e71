#!/bin/bash
# A/B over library variants, interleaved over rounds ("default" = shipped .so).
# usage: tools/abvar.sh "<workloads>" rounds V1 V2 ...   (KB_ARGS: extra kbench.py arguments, e.g. --tx)
W=$1; R=$2; shift 2
for r in $(seq $R); do
  for V in "$@"; do
    L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads $W --rounds 1 --reps 20 $KB_ARGS 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
