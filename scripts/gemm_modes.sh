#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/gemm_modes.jsonl; : > $out
for cfg in 1 0; do for ns in 2 4; do for mode in 0 1 2; do
  FD_GEMM_CFG=$cfg FD_GEMM_NS=$ns FD_GEMM_MODE=$mode timeout -k 5 120 python scripts/gemm_probe.py >> $out 2>/dev/null || exit $?
done; done; done
cat $out
