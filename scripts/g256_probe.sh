#!/bin/bash
# gemm256 (8- and 4-wave) vs gemm8 on the VAE's large-M shapes (graph-timed, scripts/gemm_probe.py)
cd "$(dirname "$0")/.."
SH="conv256x512x256x256 conv128x256x512x512 conv256x256x512x512 65536x512x4608 conv512x512x256x256"
out=gpurun_out/g256_probe.jsonl; : > $out
FD_GEMM256=1 FD_GEMM256_WAVES=8 timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?

FD_GEMM256=0 timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
cat $out
