#!/bin/bash
# r05e: halo-conv epilogue residual prefetch on the VAE's 256x128 tiles only -- A/B against the r05c build, then
# the full GPU suite and the default bench line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05e smoke "tfile=tests/test_conv_halo_gpu.py" || exit $?
for lib in fdhip/ab/libfaithdiff_hip_r05c.so fdhip/libfaithdiff_hip.so fdhip/ab/libfaithdiff_hip_r05c.so fdhip/libfaithdiff_hip.so; do
  FD_LIB_PATH=$PWD/faithdiff-dev_amd/$lib AB_TAG=$(basename $lib .so) timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/r05e_vae_ab.jsonl 2>/dev/null || exit $?
  tail -1 gpurun_out/r05e_vae_ab.jsonl | cut -c1-160
done
bash scripts/run.sh r05e tests bench || exit $?
