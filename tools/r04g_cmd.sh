# round 4: the mixed kernel's edge lines (libpnetgpu_edges.so, -DPNET_LINE_EDGES=1):
# parity suites, same-box A/B, and its IMIX read traffic (PMC FETCH_SIZE)
R=$PWD
O=$R/gpurun_out/r04g
mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_edges.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_desc_compact.py tests/test_gpu_soak.py tests/test_gpu_ext.py tests/test_gpu_tx.py -x -q --timeout 150 --timeout-method thread > $O/tests_edges.log 2>&1; rc=$?; echo edges tests rc=$rc; tail -2 $O/tests_edges.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/abvar.sh imix,imix_verify 3 default edges > $O/ab_edges.txt 2>&1; echo ab rc=$?
cd /tmp && export TMPDIR=/tmp
for V in default edges; do
  L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  PNETGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_imix_${V}_FETCH_SIZE -o run -- \
      python3 $R/tools/kbench.py --workloads imix --reps 3 --rounds 1 > $O/pmc_imix_${V}.log 2>&1 || exit 1
done
echo pmc ok
