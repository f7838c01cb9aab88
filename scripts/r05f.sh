#!/bin/bash
# r05f: VAE d=512 attention on 8 waves with split keys -- parity, then in-session A/B of the decode (FD_D512_SPLIT)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05f "tfile=tests/test_kernels_gpu.py:d512" "tfile=tests/test_pipeline_gpu.py:vae" || exit $?
for s in 0 1 0 1; do
  FD_D512_SPLIT=$s timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/r05f_vae_ab.jsonl 2>/dev/null || exit $?
  tail -1 gpurun_out/r05f_vae_ab.jsonl | cut -c1-400
done
