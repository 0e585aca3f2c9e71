#!/bin/bash
# SQ counters of slice_run_kernel on strided_probe.py shapes, per library build
# (runs on the GPU box). usage: tools/slice_pmc.sh <tag> <sizes> [lib ...]
# (lib: a PNETGPU_LIB path relative to the repo, or "default")
TAG=$1; SIZES=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in "${@:-default}"; do
  LN=$(basename $L .so)
  for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS" \
             "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
    N=$(echo $SET | cut -d' ' -f1)
    if [ "$L" = default ]; then unset PNETGPU_LIB; else export PNETGPU_LIB=$R/$L; fi
    PROBE_SIZES=$SIZES timeout -k 10 120 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $O/k${LN}_$N -o run -- \
        python3 $R/tools/strided_probe.py > $O/k${LN}_$N.log 2>&1 || { echo "pass $LN $N failed rc=$?"; exit 1; }
  done
done
python3 $R/tools/pmc_table.py $O slice_run_kernel > $O/table.txt 2>&1; cat $O/table.txt
