#!/bin/bash
# gemm256 bound diagnosis: product build vs FD_G256_DIAG builds (1 no loads, 2 load-only, 4 no epilogue)
cd "$(dirname "$0")/.."
SH="${SH:-conv128x256x512x512 conv256x512x256x256 65536x512x4608 8192x8192x8192}"
out=gpurun_out/g256_diag.jsonl; : > $out
timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
for m in 1 2 4; do
  PROBE_DIAG=$m FD_LIB_PATH=$(pwd)/faithdiff-dev_amd/fdhip/diag/lib_g$m.so timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
done
cat $out
