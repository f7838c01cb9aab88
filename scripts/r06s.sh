#!/bin/bash
# r06s: final-tree lines for the other configs: C5 (8 x 1024 px, 50 steps), C4 (8192^2 output, 225 tiles, e4m3), and
# the use_fp8 C2 step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06s "bench=--workload,c5,--no-cpu-baseline" "bench=--workload,c4,--no-cpu-baseline" \
  "bench=--fp8,--no-c3,--no-pipeline,--no-cpu-baseline"
