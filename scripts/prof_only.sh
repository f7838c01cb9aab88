#!/bin/bash
# kernel-trace profile of the bench + per-step window anatomy (no tests, no separate bench)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
name=${1:-prof_x}
bash scripts/profile.sh $name || exit $?
T=$(find gpurun_out/$name -name "*kernel_trace.csv" | head -1)
python scripts/prof_window.py $T > gpurun_out/$name/window.txt && python scripts/prof_gaps.py $T > gpurun_out/$name/gaps.txt && python scripts/roofline_check.py $T gpurun_out/$name/bench.log > gpurun_out/$name/roofline_check.json
head -24 gpurun_out/$name/window.txt
