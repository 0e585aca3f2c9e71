#!/bin/bash
# A/B over library variants x one env setting list, all workloads per variant.
# usage: tools/abenv.sh "<workloads>" "<ENV=v1,v2>" V1 V2 ...   ("default" = shipped .so)
W=$1; E=$2; shift 2
for V in "$@"; do
  L=""; [ "$V" != default ] && L=$GRAFT_REPO_ROOT/libpnet_amd/build/libpnetgpu_$V.so
  echo "== $V"
  PNETGPU_LIB=$L timeout -k 10 300 python tools/kbench.py --workloads $W --env "$E" --rounds 2 2>&1 | grep -v amdgpu.ids || exit 1
done
