#!/bin/bash
# r06h: C2 parity with the UNet in bf16 and in fp16 (the reference's UNet dtype); the fp8 GPU tests incl. the
# LayerNorm rows-per-wave bitwise test; C4 A/B: four LayerNorm rows per wave (product) vs one (build-time
# FD_LN_RPW=1, fdhip/ab/), alternated
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06h "tfile=tests/test_pipeline_gpu.py:c2_" "tfile=tests/test_fp8_gpu.py" || exit $?
AB=$PWD/faithdiff-dev_amd/fdhip/ab
OUT=gpurun_out/r06h_c4_ln_ab.txt; : > $OUT
for e in "FD_LIB_PATH=$AB/libfaithdiff_hip_ln1.so" "FD_AB_ARM=rpw4" "FD_LIB_PATH=$AB/libfaithdiff_hip_ln1.so" "FD_AB_ARM=rpw4"; do
  env $e timeout -k 10 300 python bench.py --workload c4 --steps 20 --no-cpu-baseline \
    > gpurun_out/r06h_run.json 2> gpurun_out/r06h_run.err || { echo "arm '$e' failed rc=$?"; tail -5 gpurun_out/r06h_run.err; exit 1; }
  echo "C4 $e $(tail -1 gpurun_out/r06h_run.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["c4"]; print(c["tile_steps_per_s"], c["step_ms_median"], c["latents_finite"])')" | tee -a $OUT
done
