#!/bin/bash
# Runs on the GPU box: rocprofv3 kernel-trace stats of the headline bench command
# alone (--workloads udp64: the rx_small_kernel row holds only that workload's
# launches), then of the other BASELINE workloads, then separate FETCH_SIZE /
# WRITE_SIZE PMC passes per workload and for tx_fill on tcp1500 (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950), summarised per workload by
# tools/pmc_summary.py. Output: gpurun_out/profiles_<tag>/.
set -e
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profiles_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_udp64 -o bench -- \
    python3 $R/bench.py --workloads udp64 --no-cpu --no-e2e --no-extra \
    > $O/bench_udp64_under_rocprof.json 2> $O/bench_udp64_under_rocprof.err
cp $(find $O/stats_udp64 -name "*kernel_stats.csv" | head -1) $O/kernel_stats_udp64.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_rest -o bench -- \
    python3 $R/bench.py --workloads tcp1500,imix,udp6_jumbo --no-cpu --no-e2e --no-extra \
    > $O/bench_rest_under_rocprof.json 2> $O/bench_rest_under_rocprof.err
cp $(find $O/stats_rest -name "*kernel_stats.csv" | head -1) $O/kernel_stats_tcp1500_imix_jumbo.csv
# kernel names as the library reports them (pnetgpu_last_rx_kernel, the bench line's "kernel")
declare -A KN
for W in udp64 tcp1500 imix udp6_jumbo; do
  F=$O/bench_rest_under_rocprof.json; [ $W = udp64 ] && F=$O/bench_udp64_under_rocprof.json
  KN[$W]=$(python3 -c "import json; print(json.load(open('$F'))['workloads']['$W']['kernel'])")
done
KN[tx_tcp1500]="${KN[tcp1500]%, false>}, true>"
KN[tx_udp64]="rx_small_kernel<true, false>"
for W in udp64 tcp1500 imix udp6_jumbo tx_tcp1500 tx_udp64; do
  WL=${W#tx_}; TX=""; [ "$W" != "$WL" ] && TX="--tx"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_${W}_$C -o run -- \
        python3 $R/tools/kbench.py --workloads $WL --reps 3 --rounds 1 $TX > $O/pmc_${W}_$C.log 2>&1
  done
  if [ "$W" = tx_tcp1500 ]; then
    ALG=$(python3 -c "print(1500 * 2**20 + 6 * 2**20)")
  elif [ "$W" = tx_udp64 ]; then
    ALG=$(python3 -c "print(64 * 2**24 + 6 * 2**24)")
  elif [ "$W" = udp64 ]; then
    ALG=$(python3 -c "import json; print(json.load(open('$O/bench_udp64_under_rocprof.json'))['workloads']['$W']['alg_bytes_per_launch'])" || true)
  else
    ALG=$(python3 -c "import json; print(json.load(open('$O/bench_rest_under_rocprof.json'))['workloads']['$W']['alg_bytes_per_launch'])" || true)
  fi
  python3 $R/tools/pmc_summary.py $O/pmc_${W}_FETCH_SIZE $O/pmc_${W}_WRITE_SIZE "${KN[$W]}" $O/pmc_$W.json $ALG || true
done
