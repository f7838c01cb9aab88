#!/bin/bash
# r06n: GroupNorm finalize folded into the apply kernel (producer partials) + conv_direct one channel per thread:
# kernel / halo / UNet / BSRNet / VAE-path tests, smoke, then a C2 step + VAE A/B against the two-launch GroupNorm
# (build-time FD_GN_FUSED=0, fdhip/ab/)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
AB=$PWD/faithdiff-dev_amd/fdhip/ab
bash scripts/run.sh r06n "tfile=tests/test_kernels_gpu.py" "tfile=tests/test_conv_halo_gpu.py" "tfile=tests/test_unet_gpu.py" \
  "tfile=tests/test_bsrnet_gpu.py" "tfile=tests/test_pipeline_gpu.py:vae or c2_headline" smoke \
  "abv=3;FD_LIB_PATH=$AB/libfaithdiff_hip_gn0.so;FD_AB_ARM=fused"
