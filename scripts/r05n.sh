#!/bin/bash
# r05n: output-store cache policy.  Product = sc1 write-through (FD_EPI_WT=1) on the GEMM / conv epilogues, GroupNorm
# apply, concat and flash outputs: smoke + full GPU suite on it, then the C2 step / VAE decode A/B against plain
# stores (wt0), nt (wt2) and sc1 nt (wt4), then the bench line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=$PWD/faithdiff-dev_amd/fdhip
bash scripts/run.sh r05n smoke "tests=not prescaled" || exit $?
bash scripts/run.sh r05n "abv=2;FD_LIB_PATH=$P/libfaithdiff_hip.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wt0.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wt2.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wt4.so" || exit $?
bash scripts/run.sh r05n bench || exit $?
