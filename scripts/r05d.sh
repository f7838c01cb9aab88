#!/bin/bash
# r05d: halo-conv epilogue residual prefetch -- correctness, then in-session A/B against the r05c build
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05d smoke tfile=tests/test_conv_halo_gpu.py "tfile=tests/test_pipeline_gpu.py:teacher or band" || exit $?
for lib in fdhip/ab/libfaithdiff_hip_r05c.so fdhip/libfaithdiff_hip.so fdhip/ab/libfaithdiff_hip_r05c.so fdhip/libfaithdiff_hip.so; do
  FD_LIB_PATH=$PWD/faithdiff-dev_amd/$lib timeout -k 10 300 python probes/conv_ab.py > gpurun_out/r05d_conv_ab_$(basename $lib .so).jsonl.tmp 2>&1 || exit $?
  cat gpurun_out/r05d_conv_ab_$(basename $lib .so).jsonl.tmp >> gpurun_out/r05d_conv_ab_$(basename $lib .so).jsonl; rm gpurun_out/r05d_conv_ab_$(basename $lib .so).jsonl.tmp
  FD_LIB_PATH=$PWD/faithdiff-dev_amd/$lib AB_TAG=$(basename $lib .so) timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/r05d_vae_ab.jsonl 2>/dev/null || exit $?
  tail -1 gpurun_out/r05d_vae_ab.jsonl | cut -c1-200
done
