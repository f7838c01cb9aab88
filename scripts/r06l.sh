#!/bin/bash
# r06l: final-tree rocprof evidence -- C2 bench kernel trace (step window, GEMM instances, roofline cross-check), the
# UNet GEMM-family traffic (FETCH_SIZE / WRITE_SIZE passes), the VAE decode and flash-attention counter passes -- and
# the bf16 / fp16-UNet C2 lines back to back on one box; first the halo / GroupNorm tests and smoke (fused finalize +
# affine on the statistics-pass path)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06l "tfile=tests/test_conv_halo_gpu.py" "tfile=tests/test_kernels_gpu.py:group_norm or gn" smoke "bench=--no-c3,--no-pipeline,--no-cpu-baseline" "bench=--unet-fp16,--no-c3,--no-pipeline,--no-cpu-baseline" \
  trace pmc=unet pmc=vae pmc=attn
