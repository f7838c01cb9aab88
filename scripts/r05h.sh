#!/bin/bash
# r05h: halo-conv diagnostics part 2 (18: no MFMAs and no fragment reads; 34: no K loop at all -- prologue + epilogue)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in fdhip/libfaithdiff_hip.so fdhip/ab/libfaithdiff_hip_hd18.so fdhip/ab/libfaithdiff_hip_hd34.so; do
  FD_LIB_PATH=$PWD/faithdiff-dev_amd/$lib timeout -k 10 300 python probes/conv_ab.py > gpurun_out/r05h_diag_$(basename $lib .so).jsonl 2>&1 || exit $?
done
