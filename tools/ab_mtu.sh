#!/bin/bash
# MTU tail shapes: parity of each variant on the 1500-B batch, then same-box A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03h; mkdir -p $O
for V in g16u6 g32u3 g16u6nt; do
  PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_$V.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "workload or random_frames or edge" --timeout 150 --timeout-method thread > $O/tests_$V.log 2>&1 || { echo "tests $V failed"; exit 1; }
done
echo tests ok
timeout -k 10 500 bash tools/abvar.sh tcp1500 4 default g16u6 g32u3 g16u6nt > $O/ab.txt 2>&1
echo ab rc=$?
