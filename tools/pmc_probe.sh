#!/bin/bash
# PMC comparison of rx kernel kinds on one workload (runs on the GPU box).
# usage: tools/pmc_probe.sh <workload> <kinds comma list> <tag>
W=$1; KINDS=$2; TAG=$3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $O/counters_all.txt 2>&1 || true
grep -oE "^[[:space:]]*(SQ_[A-Z_]+|TCC_[A-Z_]+|TCP_[A-Z_]+|TA_[A-Z_]+|GRBM_[A-Z_]+)" $O/counters_all.txt | sort -u > $O/counters.txt || true
for K in ${KINDS//,/ }; do
  for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM" \
             "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
    N=$(echo $SET | cut -d' ' -f1)
    PNETGPU_RX_KIND=$K timeout -k 10 200 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/k${K}_$N -o run -- \
        python3 $R/tools/kbench.py --workloads $W --reps 3 --rounds 1 > $O/k${K}_$N.log 2>&1 || echo "pass $K $N failed rc=$?"
  done
done
python3 $R/tools/pmc_table.py $O > $O/table.txt 2>&1; cat $O/table.txt
