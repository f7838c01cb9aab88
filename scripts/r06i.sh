#!/bin/bash
# r06i: halo conv ping-pong loop, first GroupNorm-transform tap (build-time FD_HALO_PP_TR: product 5; variants 2, 3 in
# fdhip/ab/): per-shape A/B of the GroupNorm-folded (and plain) UNet / VAE halo convs, alternated
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
AB=$PWD/faithdiff-dev_amd/fdhip/ab
SH="unet128_320 unet128_640to320 unet64_640 unet64_1280to640 unet64_960to640 unet64_1920to640 unet128_960to320 vae128_512 vae1024_256to128"
for v in base pptr2 pptr3 base2; do
  case $v in base|base2) lib=$PWD/faithdiff-dev_amd/fdhip/libfaithdiff_hip.so ;; *) lib=$AB/libfaithdiff_hip_$v.so ;; esac
  FD_LIB_PATH=$lib timeout -k 10 300 python -u probes/conv_ab.py $SH > gpurun_out/r06i_conv_ab_$v.jsonl 2>&1 || { tail -5 gpurun_out/r06i_conv_ab_$v.jsonl; exit 1; }
  echo "== $v"; cut -c1-150 gpurun_out/r06i_conv_ab_$v.jsonl | grep shape
done
