#!/bin/bash
# r05af: the tile-batch-bitwise tests at the new default (25, balanced), then C4 (225 tiles) with the MX activation
# forms at that batch, alternated.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05af "tfile=tests/test_configs_gpu.py:c4 or band_x4" "tfile=tests/test_tile_parallel_gpu.py:c3_49" || exit 1
OUT=gpurun_out/r05af_c4_mx_ab.txt; : > $OUT
for r in 1 2; do for e in "FD_NONE=0" "FD_FP8_MX_GEGLU=1" "FD_FP8_MX=1"; do
  env $e timeout -k 10 300 python bench.py --workload c4 --c3-steps 5 --steps 20 --no-cpu-baseline \
    > gpurun_out/r05af_run.json 2> gpurun_out/r05af_run.err || { echo "arm '$e' failed rc=$?"; tail -5 gpurun_out/r05af_run.err; exit 1; }
  echo "$e $(tail -1 gpurun_out/r05af_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c4"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"])')" | tee -a $OUT
done; done
