# round 4: lazy vs eager claims (same box, interleaved), TX write traffic of the
# whole-frame / byte-store TX against the partial / granule-store variant (PMC)
R=$PWD
O=$R/gpurun_out/r04d
mkdir -p $O
bash tools/abvar.sh udp64,udp64_verify,imix 3 default eager > $O/ab_claims.txt 2>&1; echo abclaims rc=$?
cd /tmp && export TMPDIR=/tmp
for V in default txg; do
  L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  for W in udp64 tcp1500; do
    for C in FETCH_SIZE WRITE_SIZE; do
      PNETGPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/pmc_tx_${V}_${W}_$C -o run -- \
          python3 $R/tools/kbench.py --tx --workloads $W --reps 3 --rounds 1 > $O/pmc_tx_${V}_${W}_$C.log 2>&1 || exit 1
    done
  done
done
echo pmc ok
