# round 4: jumbo shape with 32- or 16-frame runs (more waves on the same batch)
R=$PWD
O=$R/gpurun_out/r04m
mkdir -p $O
for V in jr16 jr32; do
  PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_ext.py tests/test_gpu_soak.py tests/test_gpu_sched.py -x -q --timeout 150 --timeout-method thread > $O/tests_$V.log 2>&1; rc=$?; echo $V tests rc=$rc; tail -2 $O/tests_$V.log; if [ $rc -ne 0 ]; then exit $rc; fi
done
bash tools/abvar.sh udp6_jumbo 4 default jr32 jr16 > $O/ab.txt 2>&1; echo ab rc=$?
PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_jr32.so timeout -k 10 300 python tools/kbench.py --workloads udp6_jumbo --tx --rounds 3 > $O/tx_jr32.txt 2>&1 && timeout -k 10 300 python tools/kbench.py --workloads udp6_jumbo --tx --rounds 3 > $O/tx_default.txt 2>&1; echo tx rc=$?
