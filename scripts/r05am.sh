#!/bin/bash
# r05am: the e4m3 tile planner at C4 scale (25-tile forwards, M = 51200 at the 32^2 level): default plan vs every
# launch forced to 256 x 160 or 256 x 128 (FD_F8_TILE), C4 225 tiles, 5 steps, alternated.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/r05am_f8_tile_c4_ab.txt; : > $OUT
for r in 1 2; do for e in "FD_NONE=0" "FD_F8_TILE=256160" "FD_F8_TILE=256128"; do
  env $e timeout -k 10 300 python bench.py --workload c4 --c3-steps 5 --steps 20 --no-cpu-baseline \
    > gpurun_out/r05am_run.json 2> gpurun_out/r05am_run.err || { echo "arm '$e' failed rc=$?"; tail -5 gpurun_out/r05am_run.err; exit 1; }
  echo "$e $(tail -1 gpurun_out/r05am_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c4"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"])')" | tee -a $OUT
done; done
