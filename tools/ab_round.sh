#!/bin/bash
# GPU box: interleaved A/B of library variants over several workloads, with the
# flat (kind 5) and mixed (kind 0) kernels both timed on the compact IMIX batch.
# usage: tools/ab_round.sh <tag> <rounds> <workloads> variants...
TAG=$1; R=$2; W=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq $R); do
  for V in "$@"; do
    L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads $W --rounds 1 --reps 20 2>&1 | grep -v amdgpu.ids || exit 1
    PNETGPU_LIB=$L PNETGPU_RX_KIND=0 timeout -k 10 300 python tools/kbench.py --workloads imix --rounds 1 --reps 20 2>&1 | grep -v amdgpu.ids | sed 's/^imix      /imix_mixed/' || exit 1
  done
done > $O/ab.txt 2>&1
