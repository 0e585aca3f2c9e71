#!/bin/bash
# GPU box: same-box A/B of the slice kernels (tools/slice_ab.py) over library variants.
# usage: tools/slice_ab.sh <tag> variants...   ("oldslices+grid" = oldslices with the old grid)
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  for V in "$@"; do
    L=""; E=""
    case $V in default) ;; *+grid) L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_${V%+grid}.so; E=1 ;;
                *) L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so ;; esac
    echo "== $V (round $r)"
    PNETGPU_LIB=$L PNETGPU_OLD_SLICE_GRID=$E timeout -k 10 200 python tools/slice_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt 2>&1
