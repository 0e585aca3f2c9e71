# round 4: the MTU shape with odd frames streamed backward (libpnetgpu_alt.so):
# parity suites, same-box A/B, and its 1500-B read traffic (PMC FETCH_SIZE)
R=$PWD
O=$R/gpurun_out/r04h
mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_alt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_soak.py tests/test_gpu_ext.py tests/test_gpu_tx.py -x -q --timeout 150 --timeout-method thread > $O/tests_alt.log 2>&1; rc=$?; echo alt tests rc=$rc; tail -2 $O/tests_alt.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/abvar.sh tcp1500 3 default alt > $O/ab_alt.txt 2>&1; echo ab rc=$?
cd /tmp && export TMPDIR=/tmp
for V in default alt; do
  L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  PNETGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_tcp1500_${V}_FETCH_SIZE -o run -- \
      python3 $R/tools/kbench.py --workloads tcp1500 --reps 3 --rounds 1 > $O/pmc_tcp1500_${V}.log 2>&1 || exit 1
done
echo pmc ok
