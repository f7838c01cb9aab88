#!/bin/bash
# UNet GroupNorm statistics from the producer epilogue (FD_UNET_GN_EPI=1, default) vs the GroupNorm's own
# statistics pass (=0): bench step A/B on one box, alternated.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    FD_UNET_GN_EPI=$v timeout -k 10 400 python bench.py --steps 40 --warmup 5 --no-c3 --no-pipeline --no-cpu-baseline --no-vae > gpurun_out/gnepi_$v.json 2> gpurun_out/gnepi_$v.err || exit $?
    python -c "import json,sys; d=json.loads(open('gpurun_out/gnepi_$v.json').read().strip().splitlines()[-1]); print('FD_UNET_GN_EPI=$v', d['ms_per_step'], d['forward_graph_ms'], d['kernel_ms_per_forward'])"
  done
done
