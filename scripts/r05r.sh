#!/bin/bash
# r05r: planner knob re-check on the write-through tree (every alternative that earlier rounds measured slower, now
# that the kernel-end writeback is gone): C2 step arms, then VAE-decode arms
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05r "ab=2;FD_NONE=0;FD_GEMM_R4=1;FD_GEMM_P128=1;FD_GEMM8_LNP_K=1024;FD_XATTN_GEMM=0;FD_XATTN_SPLIT=1;FD_GEMM8_MIDK=0;FD_GEMM_B4=1" || exit $?
mv gpurun_out/r05r_ab.txt gpurun_out/r05r_unet_knobs_ab.txt
bash scripts/run.sh r05r "abv=2;FD_NONE=0;FD_GEMM8_N128=1;FD_CONV_HALO=2;FD_CONV_HALO_PT=1;FD_CONV_HALO_SPLIT16=0" || exit $?
mv gpurun_out/r05r_abv.txt gpurun_out/r05r_vae_knobs_ab.txt
