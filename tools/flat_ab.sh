#!/bin/bash
# GPU box: the compact-descriptor tests, then IMIX mixed (kind 0) vs flat (kind 5)
# in one process per library variant, interleaved rounds.
# usage: tools/flat_ab.sh <tag> [variants...]   (default = the shipped .so)
set -e
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_desc_compact.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
for V in "${@:-default}"; do
  L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
  echo "== $V"
  PNETGPU_LIB=$L timeout -k 10 200 python tools/kbench.py --workloads imix --env PNETGPU_RX_KIND=0,5 --rounds 3 --reps 20
done > $O/ab.txt 2>&1
