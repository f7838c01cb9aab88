#!/bin/bash
# r05i: 256-row halo tiles with a pairwise input-channel split (FD_CONV_HALO_SPLIT16) -- halo tests, per-shape probe
# and the C2 step, both arms alternated
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05i "tfile=tests/test_conv_halo_gpu.py" "tfile=tests/test_unet_gpu.py" || exit $?
for s in 0 1; do
  FD_CONV_HALO_SPLIT16=$s timeout -k 10 300 python probes/conv_ab.py > gpurun_out/r05i_conv_ab_split16_$s.jsonl 2>&1 || exit $?
done
bash scripts/run.sh r05i "ab=2;FD_CONV_HALO_SPLIT16=0;FD_CONV_HALO_SPLIT16=1" || exit $?
