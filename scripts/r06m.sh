#!/bin/bash
# r06m: gemm8 ping-pong K loop -- GEMM / UNet / LN-fold / cross-attention GPU tests (incl. gemm256 == gemm8 bitwise and
# tile batching bitwise), smoke, then a C2 step + VAE A/B against the one-barrier loop (build-time FD_GEMM8_PP=0, fdhip/ab/)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
AB=$PWD/faithdiff-dev_amd/fdhip/ab
bash scripts/run.sh r06m "tfile=tests/test_gemm8_gpu.py" "tfile=tests/test_gemm256_gpu.py" "tfile=tests/test_unet_gpu.py" \
  "tfile=tests/test_ln_fold_gpu.py" "tfile=tests/test_xattn_gpu.py" smoke \
  "abv=3;FD_LIB_PATH=$AB/libfaithdiff_hip_pp0.so;FD_AB_ARM=pp"
