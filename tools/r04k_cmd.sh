# round 4: slice_run_kernel with descriptors one run ahead and the skipped
# word's bytes from the lane's granules (default) vs the round-3 kernel (s0)
# and the prefetch alone (pfg)
R=$PWD
O=$R/gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_packet_api.py tests/test_gpu_sched.py -x -q -k "slice or checksum" --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo tests rc=$rc; tail -2 $O/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/slice_ab.sh r04k default s0 pfg; echo ab rc=$?
