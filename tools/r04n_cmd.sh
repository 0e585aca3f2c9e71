# round 4: MTU shape with deeper group streams (U = 6, 8) at 2-4 blocks per CU
R=$PWD
O=$R/gpurun_out/r04n
mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_mtu86.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "stride or full or kat" --timeout 150 --timeout-method thread > $O/tests_mtu86.log 2>&1; rc=$?; echo tests rc=$rc; tail -1 $O/tests_mtu86.log; if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for V in default mtu86 mtu88; do
    L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads tcp1500 --env PNETGPU_BLOCKS_PER_CU=2,3,4 --rounds 2 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt 2>&1; echo ab rc=$?
