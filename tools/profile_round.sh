#!/bin/bash
# Runs on the GPU box: rocprofv3 kernel-trace stats of the default bench command,
# and separate FETCH_SIZE / WRITE_SIZE PMC passes per workload; summaries land in
# gpurun_out/profiles_<tag>/ (copy the ones to keep into profiles/).
set -e
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profiles_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- \
    python3 $R/bench.py --no-cpu --no-e2e > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
cp $O/stats/*/bench_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || cp $(find $O/stats -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
for W in udp64 tcp1500; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_${W}_$C -o run -- \
        python3 $R/tools/kbench.py --workloads $W --reps 3 --rounds 1 > $O/pmc_${W}_$C.log 2>&1
  done
done
