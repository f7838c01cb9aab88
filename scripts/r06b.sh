#!/bin/bash
# r06b: full GPU suite on the pruned library (buffer-store sc1 epilogues, ping-pong halo loop, split-K health),
# smoke, then the per-shape halo conv A/B of the ping-pong variants (build-time: transform tap PTR, setprio)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06b tests smoke || exit $?
AB=$PWD/faithdiff-dev_amd/fdhip/ab
for v in base pp60 pp40 pp51; do
  if [ $v = base ]; then lib=$PWD/faithdiff-dev_amd/fdhip/libfaithdiff_hip.so; else lib=$AB/libfaithdiff_hip_$v.so; fi
  FD_LIB_PATH=$lib timeout -k 10 300 python -u probes/conv_ab.py unet128_320 unet128_640to320 unet64_640 \
    unet64_1280to640 unet128_960to320 vae128_512 vae1024_128 vae1024_256to128 > gpurun_out/r06b_conv_ab_$v.jsonl 2>&1 || exit $?
done
