# round 4: the MTU shape's groups streaming whole 128-B lines (libpnetgpu_la.so):
# parity suites, same-box A/B, L1->L2 read requests (PMC) of both
R=$PWD
O=$R/gpurun_out/r04i
mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_la.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_soak.py tests/test_gpu_ext.py tests/test_gpu_tx.py tests/test_gpu_sched.py -x -q --timeout 150 --timeout-method thread > $O/tests_la.log 2>&1; rc=$?; echo la tests rc=$rc; tail -2 $O/tests_la.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/abvar.sh tcp1500 3 default la > $O/ab_la.txt 2>&1; echo ab rc=$?
cd /tmp && export TMPDIR=/tmp
for V in default la; do
  L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  PNETGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum --kernel-trace --output-format csv -d $O/pmc_tcp1500_${V} -o run -- \
      python3 $R/tools/kbench.py --workloads tcp1500 --reps 3 --rounds 1 > $O/pmc_tcp1500_${V}.log 2>&1 || exit 1
done
echo pmc ok
