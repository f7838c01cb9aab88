#!/bin/bash
# r05l: full GPU suite on the tree (PT auto, split16, d512 split), VAE decode A/B of the PT default (0 vs 3), bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05l smoke tests || exit $?
for r in 1 2; do for s in 0 3; do
  FD_CONV_HALO_PT=$s AB_TAG=pt$s timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/r05l_vae_ab.jsonl 2>/dev/null || exit $?
  tail -1 gpurun_out/r05l_vae_ab.jsonl | cut -c1-100
done; done
bash scripts/run.sh r05l bench || exit $?
