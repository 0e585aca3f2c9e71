#!/bin/bash
# GPU box: the round's record — GPU suite, smoke, the default bench line (the
# driver's command), then rocprofv3 stats + PMC traffic (tools/profile_round.sh).
# usage: tools/round_final.sh <tag>
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo "smoke ok"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo "bench ok"
timeout -k 10 700 bash tools/profile_round.sh $TAG > $O/profile.log 2>&1
echo "profile rc=$?"
