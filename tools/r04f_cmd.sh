# round 4: descriptor batches mixing 64-B and 9000-B frames (7:1), split tail
# items (shipped) vs whole frames per group (libpnetgpu_nosplit.so), interleaved
mkdir -p gpurun_out/r04f
for r in 1 2 3; do for V in default nosplit; do
  L=""; [ $V != default ] && L=$PWD/libpnet_amd/build/libpnetgpu_$V.so
  echo "== $V round $r" >> gpurun_out/r04f/jmix.txt
  PNETGPU_LIB=$L timeout -k 10 300 python -u tools/jmix_probe.py >> gpurun_out/r04f/jmix.txt 2>&1 || exit 1
done; done; echo jmix ok
