#!/bin/bash
# Runs on the GPU box: rocprofv3 kernel-trace stats of the bench command, one
# run per workload (each kernel_stats_<w>.csv holds only that workload's
# launches: tcp1500 and udp1500 share the MTU kernel's name), then separate
# FETCH_SIZE / WRITE_SIZE PMC passes per workload and for tx_fill (FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950), summarised per workload by
# tools/pmc_summary.py. Output: gpurun_out/profiles_<tag>/.
set -e
TAG=${1:-r05}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/profiles_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
WLS=${WLS:-udp64 tcp1500 udp1500 imix udp6_jumbo}
declare -A KN
for W in $WLS; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$W -o bench -- \
      python3 $R/bench.py --workloads $W --no-cpu --no-e2e --no-extra \
      > $O/bench_${W}_under_rocprof.json 2> $O/bench_${W}_under_rocprof.err
  cp $(find $O/stats_$W -name "*kernel_stats.csv" | head -1) $O/kernel_stats_$W.csv
  # kernel name as the library reports it (pnetgpu_last_rx_kernel, the bench line's "kernel")
  KN[$W]=$(python3 -c "import json; print(json.load(open('$O/bench_${W}_under_rocprof.json'))['workloads']['$W']['kernel'])")
done
PMC=$WLS
if [ -n "${KN[tcp1500]}" ]; then KN[tx_tcp1500]="${KN[tcp1500]%, false>}, true>"; PMC="$PMC tx_tcp1500"; fi
if [ -n "${KN[udp1500]}" ]; then KN[tx_udp1500]="${KN[udp1500]%, false>}, true>"; PMC="$PMC tx_udp1500"; fi
if [ -n "${KN[udp64]}" ]; then KN[tx_udp64]="rx_small_kernel<true, false>"; PMC="$PMC tx_udp64"; fi
for W in $PMC; do
  WL=${W#tx_}; TX=""; [ "$W" != "$WL" ] && TX="--tx"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_${W}_$C -o run -- \
        python3 $R/tools/kbench.py --workloads $WL --reps 3 --rounds 1 $TX > $O/pmc_${W}_$C.log 2>&1
  done
  if [ "$W" = tx_tcp1500 ] || [ "$W" = tx_udp1500 ]; then
    ALG=$(python3 -c "print(1500 * 2**20 + 6 * 2**20)")
  elif [ "$W" = tx_udp64 ]; then
    ALG=$(python3 -c "print(64 * 2**24 + 6 * 2**24)")
  else
    ALG=$(python3 -c "import json; print(json.load(open('$O/bench_${W}_under_rocprof.json'))['workloads']['$W']['alg_bytes_per_launch'])" || true)
  fi
  python3 $R/tools/pmc_summary.py $O/pmc_${W}_FETCH_SIZE $O/pmc_${W}_WRITE_SIZE "${KN[$W]}" $O/pmc_$W.json $ALG || true
done
