#!/bin/bash
# r06o: up-block concat writing norm1's GroupNorm statistics (fd_concat_channels_gn) + conv_direct one channel per
# thread (the fused finalize + apply of r06n measured 0.08 ms slower and is removed): kernel / UNet / C2 tests, smoke,
# then a C2 step A/B: product | FD_UNET_CAT_GN=0 | conv_direct 256 threads (build-time FD_CONV_DIRECT_MAXT=256, fdhip/ab/)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
AB=$PWD/faithdiff-dev_amd/fdhip/ab
bash scripts/run.sh r06o "tfile=tests/test_kernels_gpu.py" "tfile=tests/test_unet_gpu.py" \
  "tfile=tests/test_pipeline_gpu.py:c2_headline" smoke \
  "ab=3;FD_AB_ARM=new;FD_UNET_CAT_GN=0;FD_LIB_PATH=$AB/libfaithdiff_hip_cd256.so"
