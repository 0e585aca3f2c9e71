#!/bin/bash
# A/B over library variants, interleaved over rounds ("default" = shipped .so).
# usage: tools/abvar.sh "<workloads>" rounds V1 V2 ...   (KB_ARGS: extra kbench.py arguments, e.g. --tx;
#        AB_SCRIPT: a probe script to run per variant instead of kbench.py, e.g. tools/probes/desc_nohint_probe.py, or
#        "bench.py --workloads udp6_jumbo --no-extra --no-cpu --no-e2e" for a bench line per variant)
# Even rounds run the variants in reverse order (ABBA), so an order effect
# (the first process of a round is ~1 % slower on some boxes) cancels.
W=$1; R=$2; shift 2
FWD=("$@"); REV=(); for ((i=$#-1; i>=0; i--)); do REV+=("${FWD[$i]}"); done
for r in $(seq $R); do
  if ((r % 2)); then VS=("${FWD[@]}"); else VS=("${REV[@]}"); fi
  for V in "${VS[@]}"; do
    L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    if [ -n "$AB_SCRIPT" ]; then
      PNETGPU_LIB=$L timeout -k 10 300 python $AB_SCRIPT 2>&1 | grep -v amdgpu.ids || exit 1
    else
      PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads $W --rounds 1 --reps 20 $KB_ARGS 2>&1 | grep -v amdgpu.ids || exit 1
    fi
  done
done
