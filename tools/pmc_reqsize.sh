#!/bin/bash
# L2->fabric read requests by size (TCC_EA0_RDREQ 32B/64B/128B), per workload and
# rx kernel kind, to calibrate FETCH_SIZE on this kernel's own access pattern
# (the guide's x2 holds for 128-B streaming requests only). Runs on the GPU box.
# usage: tools/pmc_reqsize.sh <tag> <workload:kind,...>
TAG=$1; LIST=$2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/reqsize_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for WK in ${LIST//,/ }; do
  W=${WK%%:*}; K=${WK#*:}; T=k${W//_/-}-$K
  for SET in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
             "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_MISS_sum"; do
    N=$(echo $SET | cut -d' ' -f1)
    PNETGPU_RX_KIND=$K timeout -s KILL 90 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/${T}_$N -o run -- \
        python3 $R/tools/kbench.py --workloads $W --reps 3 --rounds 1 > $O/${T}_$N.log 2>&1 || { echo "pass $W $K $N failed rc=$?"; exit 1; }
  done
done
python3 $R/tools/pmc_table.py $O > $O/table.txt 2>&1; cat $O/table.txt
