#!/bin/bash
# gemm8 bound diagnosis: the same shapes with the product library and the FD_GEMM8_DIAG builds
# (1 = no operand loads, 2 = no LDS reads / MFMA: load-only, 4 = no epilogue), via FD_LIB_PATH.
cd "$(dirname "$0")/.."
SH="conv256x512x256x256 conv512x1024x128x128 262144x256x2304 65536x512x4608 conv128x256x512x512 2048x10240x1280:geglu conv64x64x640x640"
out=gpurun_out/diag_probe.jsonl; : > $out
timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
for m in 1 2 4; do
  PROBE_DIAG=$m FD_LIB_PATH=$(pwd)/faithdiff-dev_amd/fdhip/diag/lib_d$m.so timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
done
cat $out
