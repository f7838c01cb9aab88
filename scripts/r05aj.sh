#!/bin/bash
# r05aj: FD_GEMM8_LNP_BIG (large-M LN-fold producers on gemm8 256 x 160) at the tiled workloads, where the information
# transformer's producers see 25 tiles x 32768 rows: C4 (225 tiles, fp8 UNet, 5 steps) and C3 (49 tiles, bf16), alternated.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/r05aj_lnp_big_tiled_ab.txt; : > $OUT
for r in 1 2; do for e in "FD_NONE=0" "FD_GEMM8_LNP_BIG=1"; do
  env $e timeout -k 10 300 python bench.py --workload c4 --c3-steps 5 --steps 20 --no-cpu-baseline \
    > gpurun_out/r05aj_run.json 2> gpurun_out/r05aj_run.err || { echo "c4 arm '$e' failed rc=$?"; tail -5 gpurun_out/r05aj_run.err; exit 1; }
  echo "C4 $e $(tail -1 gpurun_out/r05aj_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c4"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"])')" | tee -a $OUT
  env $e timeout -k 10 300 python bench.py --workload c3 --c3-steps 10 --steps 20 --no-cpu-baseline \
    > gpurun_out/r05aj_run.json 2> gpurun_out/r05aj_run.err || { echo "c3 arm '$e' failed rc=$?"; tail -5 gpurun_out/r05aj_run.err; exit 1; }
  echo "C3 $e $(tail -1 gpurun_out/r05aj_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c3"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"])')" | tee -a $OUT
done; done
