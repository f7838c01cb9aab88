#!/bin/bash
# Targeted kernel tests, then the full GPU suite (parity metrics log), the per-shape table and the bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export FD_PARITY_METRICS=$PWD/gpurun_out/parity_metrics.json
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "groupnorm or group_norm" > gpurun_out/s_k.log 2>&1
rc=$?; tail -2 gpurun_out/s_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_suite.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/shape_table.py > gpurun_out/shape_table.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-c3 > gpurun_out/bench_suite.json 2> gpurun_out/bench_suite.err || exit $?
tail -c 600 gpurun_out/bench_suite.json
