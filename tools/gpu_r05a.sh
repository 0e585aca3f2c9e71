# round 5, first GPU pass: the new udp1500 workload (full-size parity, bench
# line, rocprof + PMC), the counter-pool scheduler and the ring's slot count
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sched.py tests/test_gpu_ring.py tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread -k "sched or ring or udp1500 or claim or streams or graph" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
echo tests ok; grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 400 python -u bench.py --workloads udp1500,tcp1500,udp64 --no-extra > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
echo bench ok
timeout -k 10 300 python -u tools/e2e_slots.py --workload udp64 --slots 3,4,6,8 > $O/e2e_slots.json 2> $O/e2e_slots.err || { echo e2e_slots failed; tail -20 $O/e2e_slots.err; exit 1; }
echo e2e ok
WLS="udp1500" timeout -k 10 400 bash tools/profile_round.sh r05a > $O/profile.log 2>&1; echo profile rc=$?
