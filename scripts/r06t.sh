#!/bin/bash
# r06t: GroupNorm statistics pass (and the concat + statistics launch) with 8 rows of loads in flight per thread
# instead of 4 (same sums, same order): kernel tests, then a C2 step + VAE A/B against U = 4 (build-time, fdhip/ab/)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
AB=$PWD/faithdiff-dev_amd/fdhip/ab
bash scripts/run.sh r06t "tfile=tests/test_kernels_gpu.py" "tfile=tests/test_unet_gpu.py" \
  "abv=3;FD_AB_ARM=u8;FD_LIB_PATH=$AB/libfaithdiff_hip_u4.so"
