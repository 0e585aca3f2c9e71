# GPU box: GPU suite, smoke(), the default bench line (the driver's command)
# usage: tools/r04_record.sh <tag>; then tools/profile_round.sh <tag> in its own call
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
echo "smoke ok"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo "bench ok"
