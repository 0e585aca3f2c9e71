#!/bin/bash
# GPU box: slice_run_kernel two-runs-at-once (slice_pair) parity + same-box A/B
# of library variants over the small-slice shapes (tools/strided_probe.py).
# usage: tools/pairs_ab.sh <tag> variants...   (default = the in-tree library)
O=gpurun_out/$1; shift
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "slice" > $O/parity_default.log 2>&1 || { echo "parity failed"; exit 1; }
for V in "$@"; do
  [ $V = default ] && continue
  PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_$V.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py \
      -x -q --timeout 120 --timeout-method thread -k "pairs or compact or dense" > $O/parity_$V.log 2>&1 \
      || { echo "parity $V failed"; exit 1; }
done
for r in 1 2; do
  for V in "$@"; do
    L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L PROBE_SIZES=${PROBE_SIZES:-20,32,48,64} timeout -k 10 200 python tools/strided_probe.py 2>&1 \
        | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt 2>&1
echo "ab rc=$?"
