#!/bin/bash
# r05k: PT halo conv, next-tile DMA after the epilogue passes (chunk 0 still prefetched in the K loop) -- tests + A/B
# tests (incl. the PT-vs-per-tile bitwise cases), then per-shape probe and VAE decode A/B, arms alternated
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05k "tfile=tests/test_conv_halo_gpu.py" || exit $?
for r in 1 2; do for s in 0 1; do
  FD_CONV_HALO_PT=$s timeout -k 10 300 python probes/conv_ab.py >> gpurun_out/r05k_conv_ab_pt$s.jsonl 2>&1 || exit $?
  FD_CONV_HALO_PT=$s AB_TAG=pt$s timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/r05k_vae_ab.jsonl 2>/dev/null || exit $?
  tail -1 gpurun_out/r05k_vae_ab.jsonl | cut -c1-120
done; done
