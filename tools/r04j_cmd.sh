# round 4: line-aligned MTU streaming at U=5 (3 rounds cover a line-padded 1500-B frame)
R=$PWD
O=$R/gpurun_out/r04j
mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_la5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tx.py -x -q --timeout 150 --timeout-method thread > $O/tests_la5.log 2>&1; rc=$?; echo la5 tests rc=$rc; tail -2 $O/tests_la5.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/abvar.sh tcp1500 3 default u5 la5 > $O/ab.txt 2>&1; echo ab rc=$?
