#!/bin/bash
# swizzled small-kernel slots: parity with the variant library, then same-box A/B
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03g; mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_swz.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_ext.py -x -q --timeout 150 --timeout-method thread > $O/tests_swz.log 2>&1
echo tests rc=$?
timeout -k 10 400 bash tools/abvar.sh udp64,udp64_verify 4 default swz > $O/ab.txt 2>&1
echo ab rc=$?
