# round 4: column stores with explicit cache-policy bits (write-through scopes)
# vs the non-temporal builtin; per-launch fixed cost of each
R=$PWD
O=$R/gpurun_out/r04l
mkdir -p $O
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_st_sys.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "not last_rx_kernel" --timeout 150 --timeout-method thread > $O/tests_sys.log 2>&1; rc=$?; echo sys tests rc=$rc; tail -2 $O/tests_sys.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/abvar.sh udp64,udp64_verify,tcp1500 2 default st_nt st_sys st_sysnt st_agent st_agentnt > $O/ab.txt 2>&1; echo ab rc=$?
for V in default st_sys st_agent; do
  L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  echo "== $V" >> $O/fixed.txt
  PNETGPU_LIB=$L timeout -k 10 300 python tools/launch_fixed.py udp64,tcp1500 >> $O/fixed.txt 2>&1 || exit 1
done
echo fixed ok
