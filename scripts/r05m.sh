#!/bin/bash
# r05m: epilogue store cache policy A/B (plain / sc1 write-through / nt) on the C2 step and the VAE decode, and a
# flash-attention timing build without K/V loads after the prologue (FD_FLASH_DIAG=1: how much of the kernel the
# loads take)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=$PWD/faithdiff-dev_amd/fdhip
bash scripts/run.sh r05m "abv=2;FD_LIB_PATH=$P/libfaithdiff_hip.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wt1.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wt2.so" || exit $?
for lib in libfaithdiff_hip.so ab/libfaithdiff_hip_fd1.so; do
  FD_LIB_PATH=$P/$lib timeout -k 10 200 python scripts/attn_probe.py > gpurun_out/r05m_attn_$(basename $lib .so).jsonl 2>&1 || exit $?
  cat gpurun_out/r05m_attn_$(basename $lib .so).jsonl
done
