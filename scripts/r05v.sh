#!/bin/bash
# r05v: final-tree counter passes -- flash attention (SQ VALU / MFMA / LDS groups) and the VAE decode (L2-miss traffic
# of the convs, GroupNorm bandwidth) on the write-through tree
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05v pmc=attn pmc=vae || exit $?
