#!/bin/bash
# Same-box A/B of the ring's descriptor form: the shipped library (compact
# u32/u16 descriptors) vs a build that always ships u64/u32 ones
# (-DPNETGPU_RING_FULL_DESC). Build here first:
#   make -C libpnet_amd && (cd libpnet_amd && hipcc -O3 -std=c++17 -fPIC -I../include -Icsrc \
#     -DPNETGPU_RING_FULL_DESC -c csrc/ring.cpp -o build/ring_full.o && hipcc --offload-arch=gfx950 -shared \
#     -fPIC -o build/libpnetgpu_fulldesc.so build/rx_kernel.o build/abi.o build/synth.o build/ring_full.o \
#     build/afpacket.o -lpthread)
R=${1:-2}
for r in $(seq $R); do
  for V in default fulldesc; do
    L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
    echo "== $V (round $r)"
    PNETGPU_LIB=$L timeout -k 10 200 python bench.py --workloads udp64 --no-cpu --no-extra --steps 5 --warmup 2 \
      | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print({k: d[k] for k in ('e2e_pcie','e2e_ring','e2e_zero_copy')})" || exit 1
  done
done
