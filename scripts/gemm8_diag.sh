#!/bin/bash
# gemm8 diagnostics: load-only / compute-only / no-epilogue timings vs full, and one SQ PMC pass.
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out/diag
out=gpurun_out/diag/modes.jsonl; : > $out
SH="32768x1920x640 2048x1280x5120 2048x10240x1280:geglu conv32x32x1280x1280"
for m in 0 1 2 4 6; do
  FD_GEMM8_S=1 FD_GEMM8_MODE=$m timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>>gpurun_out/diag/err.log || exit $?
done
FD_GEMM8=0 timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>>gpurun_out/diag/err.log || exit $?
cat $out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/diag/counters.txt 2>&1 || true
cd /tmp
for k in 1 0; do
  FD_GEMM8=$k FD_GEMM8_S=1 PROBE_REP=4 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS \
    --output-format csv -d $R/gpurun_out/diag/pmc$k -o run -- python3 $R/scripts/gemm_probe.py 32768x1920x640 > $R/gpurun_out/diag/pmc$k.log 2>&1 || exit $?
done
