#!/bin/bash
# SQ counter passes over the flash kernel (one pass per counter group, kernel-trace only)
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/apmc
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/apmc/counters.txt 2>&1) || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1)); d=$R/gpurun_out/apmc/p$i
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $d -o run \
     -- python3 $R/scripts/attn_pmc_run.py > $R/gpurun_out/apmc/p$i.log 2>&1)
  echo "pass $i rc=$?"; tail -2 $R/gpurun_out/apmc/p$i.log
done
find gpurun_out/apmc -name "*counter_collection*" | head
