#!/bin/bash
# PMC passes over the C2 flash-attention shapes (attn_probe.py: graph-replayed launches): is the d64 kernel bound by
# the LDS array (SQ_LDS_IDX_ACTIVE vs GRBM_GUI_ACTIVE), MFMA, VALU issue or waits?
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/attn_pmc3; rm -rf $o; mkdir -p $o
run() {  # $1 = pass name, rest = counters
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --stats -d $o/$n -o run -- python scripts/attn_probe.py 2x20x1024x1024 2x10x4096x4096 > $o/$n.log 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU && \
run p2 GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU && \
run p3 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM || exit $?
for p in p1 p2 p3; do for db in $(find $o/$p -name "*.db"); do python scripts/rocpd_pmc.py $db --filter flash; done; done
