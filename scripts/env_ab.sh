#!/bin/bash
# in-step A/B of env knobs: bench ms/step (no CPU baseline, no VAE), alternating arms twice
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/env_ab.txt; : > $out
for rep in 1 2; do
for e in "X=0" "$@"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-vae --steps 30 > gpurun_out/env_ab_run.log 2>&1 || exit $?
  echo "$e $(tail -1 gpurun_out/env_ab_run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a $out
done; done
