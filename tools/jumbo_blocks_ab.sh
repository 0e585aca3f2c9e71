set -o pipefail
mkdir -p gpurun_out/jumbo_blocks
for i in 1 2; do for V in default jb4; do for s in 1 2 4; do
  L=""; [ $V != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
  PNETGPU_LIB=$L timeout -k 10 200 python bench.py --workloads udp6_jumbo --no-extra --no-cpu --no-e2e --frames-scale $s 2>/dev/null | python3 -c "import json,sys; b=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$V', $s, b['config']['frames_per_gpu'], b['roofline']['frac'], b['ms_per_step'])" || exit 1
done; done; done
