#!/bin/bash
# Runs on the GPU box: FETCH_SIZE / WRITE_SIZE passes for the IMIX workload as
# bench.py now runs it (compact descriptors), summarised into
# profiles/pmc_imix.json (read by bench.py for roofline.traffic), then the
# default bench line and its rocprofv3 --stats run. Output: gpurun_out/final/.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
ALG=${1:?algorithmic bytes per IMIX launch}
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_imix_$C -o run -- \
      python3 $R/tools/kbench.py --workloads imix --reps 3 --rounds 1 > $O/pmc_imix_$C.log 2>&1
done
python3 $R/tools/pmc_summary.py $O/pmc_imix_FETCH_SIZE $O/pmc_imix_WRITE_SIZE \
    "rx_kernel<8, 4, 8, false, 0, true, false, false" $O/pmc_imix.json $ALG
cp $O/pmc_imix.json $R/profiles/pmc_imix.json
cd $R
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- \
    python3 $R/bench.py --no-cpu --no-e2e > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err
cp $(find $O/stats -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
