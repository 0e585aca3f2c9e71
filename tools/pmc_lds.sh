#!/bin/bash
# LDS and VALU counters of the default kernel per workload (runs on the GPU box).
# usage: tools/pmc_lds.sh <tag> <workloads comma list>
TAG=$1; WS=$2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for W in ${WS//,/ }; do
  for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY"; do
    N=$(echo $SET | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/k${W}_$N -o run -- \
        python3 $R/tools/kbench.py --workloads $W --reps 3 --rounds 1 > $O/k${W}_$N.log 2>&1 || echo "pass $W $N failed rc=$?"
  done
done
python3 $R/tools/pmc_table.py $O > $O/table.txt 2>&1; cat $O/table.txt
