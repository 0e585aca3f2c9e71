#!/bin/bash
# GPU box: SQ/LDS counters of the split kernel (kind 6) on one workload, per
# library variant. usage: tools/pmc_split.sh <tag> <workload> variants...
TAG=$1; W=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  L=""; [ "$V" != default ] && L=$R/libpnet_amd/build/libpnetgpu_$V.so
  for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
    N=$(echo $SET | cut -d' ' -f1)
    PNETGPU_LIB=$L PNETGPU_RX_KIND=6 timeout -s KILL 90 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/k${V}_$N -o run -- \
        python3 $R/tools/kbench.py --workloads $W --reps 3 --rounds 1 > $O/k${V}_$N.log 2>&1 || { echo "pass $V $N failed"; exit 1; }
  done
done
python3 $R/tools/pmc_table.py $O > $O/table.txt 2>&1; cat $O/table.txt
