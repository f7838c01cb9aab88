#!/bin/bash
# r05ad: C4 (225 tiles at 8192^2 output, use_fp8) tile-steps/s against the tile batching (FD_TILE_BATCH /
# FD_TILE_BALANCE), arms alternated, 5 Euler steps per run after the 1-step warm-up.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/r05ad_tile_batch_ab.txt; : > $OUT
ARMS=("FD_NONE=0" "FD_TILE_BALANCE=1" "FD_TILE_BATCH=15" "FD_TILE_BATCH=19 FD_TILE_BALANCE=1" "FD_TILE_BATCH=25")
for r in 1 2; do for e in "${ARMS[@]}"; do
  env $e timeout -k 10 300 python bench.py --workload c4 --c3-steps 5 --steps 20 --no-cpu-baseline \
    > gpurun_out/r05ad_run.json 2> gpurun_out/r05ad_run.err || { echo "arm '$e' failed rc=$?"; tail -5 gpurun_out/r05ad_run.err; exit 1; }
  echo "$e $(tail -1 gpurun_out/r05ad_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c4"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"])')" | tee -a $OUT
done; done
