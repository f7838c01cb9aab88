#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/gemm_sweep.jsonl
: > $OUT
for swz in 0 1; do
 for ns in 2 3 4; do
  for cfg in -1 0 1 2; do
    FD_GEMM_CFG=$cfg FD_GEMM_NS=$ns FD_GEMM_SWZ=$swz timeout -k 10 120 python scripts/gemm_sweep.py >> $OUT 2> gpurun_out/gemm_sweep.err
    rc=$?; if [ $rc -ne 0 ]; then echo "rc=$rc cfg=$cfg ns=$ns swz=$swz"; tail -3 gpurun_out/gemm_sweep.err; exit $rc; fi
  done
 done
done
wc -l $OUT
