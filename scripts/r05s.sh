#!/bin/bash
# r05s: the 32^2 ff-out producer forms on the write-through tree (256 x 160 with an S-way K split, the 4-wave 64 x 160
# producer) against the default 128 x 160 pairwise split
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05s "ab=2;FD_NONE=0;FD_GEMM8_LNP=2;FD_GEMM8_LNP=2 FD_GEMM8_LNP_S=2;FD_GEMM8_LNP=0" || exit $?
# GELU cost in the GEGLU epilogue: timing build that multiplies by g instead of gelu(g) (FD_GEGLU_DIAG=1, wrong results)
P=$PWD/faithdiff-dev_amd/fdhip
bash scripts/run.sh r05s_gd "ab=2;FD_LIB_PATH=$P/libfaithdiff_hip.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_gd1.so" || exit $?
