# round 4: line-aligned MTU streaming at U=5 (3 rounds cover a line-padded 1500-B frame)
R=$PWD
O=$R/gpurun_out/r04j
mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_la5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tx.py -x -q -k "not last_rx_kernel" --timeout 150 --timeout-method thread > $O/tests_la5.log 2>&1; rc=$?; echo la5 tests rc=$rc; tail -2 $O/tests_la5.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/abvar.sh tcp1500 3 default u5 la5 > $O/ab.txt 2>&1; echo ab rc=$?
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_mla11.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_desc_compact.py tests/test_gpu_soak.py tests/test_gpu_ext.py tests/test_gpu_tx.py -x -q --timeout 150 --timeout-method thread > $O/tests_mla11.log 2>&1; rc=$?; echo mla11 tests rc=$rc; tail -2 $O/tests_mla11.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/abvar.sh imix,imix_verify 3 default mla11 mla12 > $O/ab_mla.txt 2>&1; echo abmla rc=$?
cd /tmp && export TMPDIR=/tmp
for V in default mla11; do
  L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  PNETGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum --kernel-trace --output-format csv -d $O/pmcreq_imix_${V} -o run -- \
      python3 $R/tools/kbench.py --workloads imix --reps 3 --rounds 1 > $O/pmcreq_imix_${V}.log 2>&1 || exit 1
  PNETGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmcfetch_imix_${V} -o run -- \
      python3 $R/tools/kbench.py --workloads imix --reps 3 --rounds 1 > $O/pmcfetch_imix_${V}.log 2>&1 || exit 1
done
echo pmc ok
