#!/bin/bash
cd "$(dirname "$0")/.."
out=gpurun_out/gemm_modes2.jsonl; : > $out
for cfg in 0 1; do for mode in 0 1 2; do
  FD_GEMM_CFG=$cfg FD_GEMM_MODE=$mode timeout -k 5 120 python scripts/gemm_probe.py 8192x5120x1280 2048x10240x1280 32768x1920x640 2048x1280x5120 >> $out 2>/dev/null || exit $?
done; done
cat $out
