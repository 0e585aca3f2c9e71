#!/bin/bash
# GPU box: same-box A/B of short-run granule loads, in-tree library vs a variant (usage: <tag> <variant>)
O=gpurun_out/$1; shift
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k short \
    > $O/parity.log 2>&1 || { echo "parity failed"; exit 1; }
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_$1.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q \
    --timeout 120 --timeout-method thread -k short >> $O/parity.log 2>&1 || { echo "parity nt failed"; exit 1; }
for r in 1 2 3; do
  for V in default "$@"; do
    L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L timeout -k 10 200 python tools/desc64_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
    PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads imix --rounds 1 --reps 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt 2>&1
echo "ab rc=$?"
