#!/bin/bash
# r05ae: larger tile batches.  (1) the C4 literal reading (1947 tiles, 1 step) with 25-tile balanced batches: rate and
# peak HBM; (2) the C3 leg of the default bench (49 tiles, bf16) with 13 vs 25 balanced, alternated.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
env FD_TILE_BATCH=25 FD_TILE_BALANCE=1 timeout -k 10 400 python -u scripts/c4_literal.py --steps 1 \
  > gpurun_out/r05ae_c4_literal_tb25.log 2>&1 || { echo "c4 literal failed rc=$?"; tail -5 gpurun_out/r05ae_c4_literal_tb25.log; exit 1; }
tail -1 gpurun_out/r05ae_c4_literal_tb25.log
OUT=gpurun_out/r05ae_c3_tile_batch_ab.txt; : > $OUT
for r in 1 2; do for e in "FD_NONE=0" "FD_TILE_BATCH=25 FD_TILE_BALANCE=1"; do
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-vae --no-pipeline --steps 10 \
    > gpurun_out/r05ae_run.json 2> gpurun_out/r05ae_run.err || { echo "arm '$e' failed rc=$?"; tail -5 gpurun_out/r05ae_run.err; exit 1; }
  echo "$e $(tail -1 gpurun_out/r05ae_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c3"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"], c["s_per_image"])')" | tee -a $OUT
done; done
