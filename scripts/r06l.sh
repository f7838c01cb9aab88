#!/bin/bash
# r06l: final-tree rocprof evidence: C2 bench kernel trace (step window, GEMM instances, roofline cross-check), the UNet
# GEMM-family traffic (FETCH_SIZE / WRITE_SIZE passes), the VAE decode and flash-attention counter passes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06l trace pmc=unet pmc=vae pmc=attn
