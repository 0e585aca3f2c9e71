#!/bin/bash
# One GPU call = a list of named steps, each under its own time limit, chained:
# the call stops at the first failing step (no retries). Output under
# gpurun_out/<TAG>/. Replaces the single-use per-call scripts of earlier rounds.
#
#   bash tools/gpu_steps.sh TAG STEP [STEP ...]
#
# STEP is one of
#   suite                      the whole GPU suite (pytest -m gpu)
#   tests:FILE[+FILE...][:K]   those test files, -m gpu, optionally -k K ('+' for spaces)
#   smoke                      __graft_entry__.smoke()
#   bench[:W,W...]             bench.py (default workloads, or --workloads W,.. --no-extra)
#   profile[:W+W...]           tools/profile_round.sh (rocprofv3 stats + PMC) for those workloads
#   variant:V:K[:FILE+FILE]    tests/test_gpu_parity.py (or FILEs) -k K on libpnetgpu_V.so (PNETGPU_LIB)
#   ab:W:ROUNDS:V+V...         tools/abvar.sh interleaved A/B of library variants (KB_ARGS passes through)
#   e2e:W:SLOTS                tools/e2e_slots.py (ring slot sweep, e.g. 3,4,6)
#   py:SCRIPT[:ARGS]           python -u SCRIPT ARGS ('+' for spaces), output in the step log
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
R=${GRAFT_REPO_ROOT:-$(pwd)}
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
n=0
for S in "$@"; do
  n=$((n + 1))
  IFS=: read -r K A1 A2 A3 <<< "$S"
  L=$O/$(printf %02d $n)_$K.log
  case $K in
    suite) timeout -k 10 900 $PYT tests -m gpu > $L 2>&1 ;;
    tests) A2=${A2//+/ }; timeout -k 10 600 $PYT ${A1//+/ } -m gpu ${A2:+-k "$A2"} > $L 2>&1 ;;
    smoke) timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $L 2>&1 ;;
    bench) if [ -n "$A1" ]; then
             timeout -k 10 500 python -u bench.py --workloads $A1 --no-extra > $O/bench_$n.json 2> $L
           else
             timeout -k 10 600 python -u bench.py > $O/bench.json 2> $L
           fi ;;
    profile) WLS="${A1//+/ }" timeout -k 10 900 bash tools/profile_round.sh $TAG > $L 2>&1 ;;
    variant) A2=${A2//+/ }; A3=${A3//+/ }; PNETGPU_LIB=$R/libpnet_amd/build/libpnetgpu_$A1.so timeout -k 10 400 \
               $PYT ${A3:-tests/test_gpu_parity.py} -k "$A2" > $L 2>&1 ;;
    ab) timeout -k 10 1200 bash tools/abvar.sh $A1 $A2 ${A3//+/ } > $L 2>&1 ;;
    e2e) timeout -k 10 400 python -u tools/e2e_slots.py --workload $A1 --slots $A2 > $O/e2e_$A1.json 2> $L ;;
    py) timeout -k 10 600 python -u $A1 ${A2//+/ } > $L 2>&1 ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
  rc=$?
  echo "step $n $S rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 $L; exit $rc; fi
  grep -E "passed|failed" $L 2>/dev/null | tail -1 || true
done
