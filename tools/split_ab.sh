#!/bin/bash
# GPU box: the split kernel (kind 6) against each workload's default kernel, in
# one process per workload (interleaved rounds), for the default build and the
# ring-depth variants given as arguments.
# usage: tools/split_ab.sh <tag> variants...
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for V in "$@"; do
  L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
  echo "== $V"
  for WK in imix:0 tcp1500:2 udp6_jumbo:3 imix_verify:0; do
    W=${WK%%:*}; K=${WK#*:}
    PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads $W --env PNETGPU_RX_KIND=$K,6 --rounds 3 --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt 2>&1
