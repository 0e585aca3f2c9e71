# Jumbo-workload bench fractions at 2^17 / 2^18 / 2^19 frames per library variant
# ("default" = the shipped .so), two interleaved rounds.
# usage: tools/jumbo_blocks_ab.sh [V1 V2 ...]   (default: default jb4)
set -o pipefail
mkdir -p gpurun_out/jumbo_blocks
VS=${*:-default jb4}
for i in 1 2; do for V in $VS; do for s in 1 2 4; do
  L=""; [ $V != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
  PNETGPU_LIB=$L timeout -k 10 200 python bench.py --workloads udp6_jumbo --no-extra --no-cpu --no-e2e --frames-scale $s 2>/dev/null | python3 -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$V', $s, b['config']['frames_per_gpu'], b['roofline']['frac'], b['ms_per_step'])" || exit 1
done; done; done
