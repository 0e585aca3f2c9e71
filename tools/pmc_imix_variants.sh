R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for V in ${VARIANTS:-default}; do
  L=""; [ $V != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  PNETGPU_LIB=$L timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcimix_$V -o run -- python3 $R/tools/kbench.py --workloads imix --reps 3 --rounds 1 > $R/gpurun_out/pmcimix_$V.log 2>&1 || exit 1
  python3 - $R/gpurun_out/pmcimix_$V <<'PY'
import csv,glob,sys,statistics
v=[float(r["Counter_Value"]) for f in glob.glob(sys.argv[1]+"/**/*counter_collection.csv",recursive=True) for r in csv.DictReader(open(f)) if r["Counter_Name"]=="FETCH_SIZE" and "rx_kernel" in r["Kernel_Name"]]
print(sys.argv[1].split("_")[-1], "FETCH_SIZE x2 bytes/launch", statistics.median(v)*2048 if v else None)
PY
done
