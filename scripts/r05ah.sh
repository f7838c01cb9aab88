#!/bin/bash
# r05ah: (1) the default bench line again (box-to-box spread of the final tree); (2) epilogue / operand-load share of
# the 16-bit GEMM shapes: product library vs -DFD_GEMM8_DIAG=4 (no epilogue stores) vs =1 (no operand loads),
# graph-timed per launch (scripts/gemm_probe.py; diagnostic builds are timing-only, their outputs are wrong).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05ah bench || exit $?
out=gpurun_out/r05ah_epi_share.jsonl; : > $out
SH="2048x1280x1280 2048x1280x5120 2048x3840x1280 2048x10240x1280:geglu 8192x640x640 8192x640x2560 32768x320x320"
for lib in product d4 d1; do
  if [ $lib = product ]; then unset FD_LIB_PATH; else export FD_LIB_PATH=$PWD/faithdiff-dev_amd/fdhip/ab/libfaithdiff_hip_$lib.so; fi
  PROBE_TAG=$lib timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>gpurun_out/r05ah_probe.err || { echo "probe $lib failed"; tail -3 gpurun_out/r05ah_probe.err; exit 1; }
done
cat $out
