#!/bin/bash
# Memory-pipeline counters of each workload's default kernel (GPU box): L1->L2
# read requests and their latency, address-translation (UTCL1) misses, TA/TD
# busy and stalls, L2->fabric read level (Little's law: latency) and DRAM credit
# stalls, wave waits. One rocprofv3 --pmc pass per counter set (block limits:
# 4 TCP, 2 TA, 2 TD, 4 TCC, 8 SQ, 2 GRBM), summed per dispatch by pmc_table.py.
# usage: tools/pmc_mem.sh <tag> <workloads comma list>
TAG=$1; WS=$2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcmem_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for W in ${WS//,/ }; do
  for SET in "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_HIT_sum" \
             "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
             "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum" \
             "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES"; do
    N=$(echo $SET | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/k${W}_$N -o run -- \
        python3 $R/tools/kbench.py --workloads $W --reps 3 --rounds 1 > $O/k${W}_$N.log 2>&1 || { echo "pass $W $N failed rc=$?"; exit 1; }
  done
done
python3 $R/tools/pmc_table.py $O > $O/table.txt 2>&1; cat $O/table.txt
