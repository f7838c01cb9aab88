#!/bin/bash
# r05an: the e4m3 planner's large-M rule (256 x 128 for M >= 16384): fp8 GPU tests, the C4 tile-batch-bitwise test,
# smoke, then C4 default vs forced 256 x 128 (should now be equal) and the use_fp8 C2 step (unchanged plan), alternated.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05an smoke tfile=tests/test_fp8_gpu.py "tfile=tests/test_configs_gpu.py:c4" || exit 1
OUT=gpurun_out/r05an_f8_rule_ab.txt; : > $OUT
for e in "FD_NONE=0" "FD_F8_TILE=256128" "FD_NONE=0"; do
  env $e timeout -k 10 300 python bench.py --workload c4 --c3-steps 5 --steps 20 --no-cpu-baseline \
    > gpurun_out/r05an_run.json 2> gpurun_out/r05an_run.err || { echo "arm '$e' failed rc=$?"; tail -5 gpurun_out/r05an_run.err; exit 1; }
  echo "C4 $e $(tail -1 gpurun_out/r05an_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c4"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"])')" | tee -a $OUT
done
