#!/bin/bash
# flash d64: how the L = 1024 launch time splits into per-tile work and fixed cost (Lk, Lq, heads scaled)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/attn_scale.jsonl; : > $out
S="2x20x1024x1024 2x20x1024x512 2x20x1024x2048 2x20x1024x4096 2x20x2048x1024 2x40x1024x1024 4x40x1024x1024 2x10x4096x4096"
for w in 4 2; do
  FD_FLASH_WAVES=$w timeout -k 10 120 python scripts/attn_probe.py $S >> $out 2>/dev/null || exit $?
done
cat $out
