# round 5, second GPU pass: ring push fix + netns loopback legs (default build),
# then the IMIX occupancy question: NW=6 (5 waves/SIMD) variants, parity first,
# then a same-box interleaved A/B against the shipped NW=8
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_netns_loopback.py tests/test_pcapdump.py -x -v --timeout 200 --timeout-method thread -m gpu -s > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
echo tests ok; grep -E "passed|failed|skipped" $O/tests.log | tail -3
PNETGPU_LIB=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_nw6u8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "imix and full_size" > $O/parity_nw6u8.log 2>&1 || { echo nw6 parity failed; tail -30 $O/parity_nw6u8.log; exit 1; }
echo nw6 parity ok
timeout -k 10 900 bash tools/abvar.sh imix 3 default nw6u8 nw6u6 nw6u4 > $O/ab_nw6.txt 2>&1 || { echo ab failed; tail -20 $O/ab_nw6.txt; exit 1; }
echo ab ok
timeout -k 10 300 python -u tools/e2e_slots.py --workload udp1500 --slots 3,4 > $O/e2e_slots_udp1500.json 2> $O/e2e_slots_udp1500.err || { echo e2e failed; tail -20 $O/e2e_slots_udp1500.err; exit 1; }
echo e2e ok
