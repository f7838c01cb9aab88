#!/bin/bash
# r05u: GEGLU epilogue on packed f32 VALU (gelu2_f): GEGLU / LN-fold GPU tests + UNet parity, then the C2 step A/B
# against the scalar-epilogue library
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=$PWD/faithdiff-dev_amd/fdhip
bash scripts/run.sh r05u "tfile=tests/test_gemm8_gpu.py" "tfile=tests/test_kernels_gpu.py:geglu or gemm" "tfile=tests/test_unet_gpu.py" || exit $?
bash scripts/run.sh r05u "ab=3;FD_LIB_PATH=$P/libfaithdiff_hip.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_gelu_scalar.so" || exit $?
