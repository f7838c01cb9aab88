#!/bin/bash
# PMC passes over the ping-pong probe's full kernel and its single-path variants (2048 x 10240 x 1280, 256 x 160).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
o=gpurun_out/pp_pmc; rm -rf $o; mkdir -p $o
run() {  # $1 = pass name, rest = counters
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --stats -d $o/$n -o run -- ./probes/gemm_pp faithdiff-dev_amd/fdhip/libfaithdiff_hip.so pmc > $o/$n.log 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS && \
run p2 GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU && \
run p3 TA_TA_BUSY_sum TA_BUSY_avr SQ_INST_CYCLES_VMEM SQ_INSTS_VALU
ls -R $o | head -50
