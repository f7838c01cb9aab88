#!/bin/bash
# Share of gemm8's epilogue in the UNet's eight-wave launches: the product library vs a build with
# -DFD_GEMM8_DIAG=4 (main loop + split-K combine, no epilogue stores), each with FD_GEMM_PP=0/1.
cd "$(dirname "$0")/.."
out=gpurun_out/epi_share.jsonl; : > $out
SH="2048x10240x1280:geglu 2048x10240x1280 2048x3840x1280 8192x5120x640:geglu conv128x128x320x320 conv64x64x640x640 conv32x32x1280x1280"
for lib in product diag4; do for pp in 0 1; do
  if [ $lib = diag4 ]; then export FD_LIB_PATH=$PWD/probes/lib_g8diag4.so; else unset FD_LIB_PATH; fi
  FD_GEMM_PP=$pp PROBE_TAG=$lib timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
done; done
cat $out
