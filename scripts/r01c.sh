#!/bin/bash
# round-1 measurement pass: kernel parity subset, bench (N=1), kernel-trace profile + per-step window/gap anatomy
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_gemm8_gpu.py -m gpu -x -q -p no:cacheprovider > gpurun_out/kern.log 2>&1
rc=$?; tail -1 gpurun_out/kern.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r01c.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r01c.log
bash scripts/profile.sh prof_r01c || exit $?
T=$(find gpurun_out/prof_r01c -name "*kernel_trace.csv" | head -1)
python scripts/prof_window.py $T > gpurun_out/prof_r01c/window.txt && python scripts/prof_gaps.py $T > gpurun_out/prof_r01c/gaps.txt && python scripts/roofline_check.py $T gpurun_out/prof_r01c/bench.log > gpurun_out/prof_r01c/roofline_check.json
head -20 gpurun_out/prof_r01c/window.txt
