#!/bin/bash
# GPU box: slice_tiny_kernel of library variants ("default" = shipped .so),
# interleaved rounds, through tools/tiny_probe.py.
# usage: tools/tiny_ab.sh TAG SIZES V1 V2 ...
O=gpurun_out/$1; Z=$2; shift 2
mkdir -p $O
for r in 1 2 3; do
  for V in "$@"; do
    L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L timeout -k 10 200 python tools/tiny_probe.py --sizes $Z --rounds 1 --variants tiny 2>&1 \
      | grep -v amdgpu.ids || exit 1
  done
done > $O/tiny_ab.txt 2>&1
