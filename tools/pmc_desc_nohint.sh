#!/bin/bash
# HBM traffic (FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 --pmc passes) of
# the mixed kernel on a no-hint descriptor batch of fixed-size frames, per
# library variant ("default" = the shipped .so).
# usage: tools/pmc_desc_nohint.sh <udp1500|udp6_jumbo> <tag> V1 V2 ...
W=$1; TAG=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_nohint_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ALG=$(python3 -c "n={'udp1500':1<<20,'udp6_jumbo':1<<17}['$W']; f={'udp1500':1500,'udp6_jumbo':9000}['$W']; print(n*(f+32))")
for V in "$@"; do
  L=""; [ "$V" != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  for C in FETCH_SIZE WRITE_SIZE; do
    PNETGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/${V}_$C -o run -- \
      python3 $R/tools/desc_nohint_probe.py --nohint-only $W > $O/${V}_$C.log 2>&1 || { echo "pass $V $C failed"; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $O/${V}_FETCH_SIZE $O/${V}_WRITE_SIZE "rx_kernel<8, 4, 8" $O/${V}.json $ALG
  echo "== $V"; cat $O/${V}.json; echo
done
