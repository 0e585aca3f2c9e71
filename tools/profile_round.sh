#!/bin/bash
# Runs on the GPU box: rocprofv3 kernel-trace stats of the bench command over all
# four BASELINE workloads, then separate FETCH_SIZE / WRITE_SIZE PMC passes per
# workload (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), summarised
# per workload by tools/pmc_summary.py. Output: gpurun_out/profiles_<tag>/.
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profiles_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- \
    python3 $R/bench.py --workloads udp64,tcp1500,imix,udp6_jumbo --no-cpu --no-e2e \
    > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
cp $(find $O/stats -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
declare -A KN=([udp64]=rx_small_kernel [tcp1500]="rx_kernel<8, 8, 4, false, 1, false, false, false" [imix]="rx_kernel<8, 4, 8, false, 0, true, false, false" [udp6_jumbo]="rx_kernel<8, 64, 9, true, 0, false, false, false")
for W in udp64 tcp1500 imix udp6_jumbo; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_${W}_$C -o run -- \
        python3 $R/tools/kbench.py --workloads $W --reps 3 --rounds 1 > $O/pmc_${W}_$C.log 2>&1
  done
  ALG=$(python3 -c "import json; print(json.load(open('$O/bench_under_rocprof.json'))['workloads']['$W']['alg_bytes_per_launch'])" || true)
  python3 $R/tools/pmc_summary.py $O/pmc_${W}_FETCH_SIZE $O/pmc_${W}_WRITE_SIZE "${KN[$W]}" $O/pmc_$W.json $ALG || true
done
