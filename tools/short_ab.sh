#!/bin/bash
# GPU box: the mixed kernel's short-run path — parity, then a same-box A/B
# (tools/desc64_probe.py: 64-B frames over descriptors; tools/kbench.py: IMIX and
# MTU) of the in-tree library against library variants. usage: tools/short_ab.sh <tag> variants...
O=gpurun_out/$1; shift
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ring.py tests/test_gpu_sched.py -x -q \
    --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || { echo "parity failed"; tail -30 $O/parity.log; exit 1; }
echo "parity ok"
for r in 1 2; do
  for V in default "$@"; do
    L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L timeout -k 10 200 python tools/desc64_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
    PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads imix,tcp1500,udp64 --rounds 1 --reps 20 2>&1 \
        | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt 2>&1
echo "ab rc=$?"
