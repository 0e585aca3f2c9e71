# round 4: the verify-only record against its skeletons on one box (sol5),
# then the bench's small-kernel lines in the same call
mkdir -p gpurun_out/r04e
timeout -k 10 200 ./tools/sol5 r > gpurun_out/r04e/sol5.txt 2>&1; echo sol5 rc=$?
timeout -k 10 300 python -u tools/kbench.py --workloads udp64,udp64_verify --rounds 3 --reps 20 > gpurun_out/r04e/kb.txt 2>&1; echo kb rc=$?
timeout -k 10 200 ./tools/sol5 r >> gpurun_out/r04e/sol5.txt 2>&1; echo sol5b rc=$?
