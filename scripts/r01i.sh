#!/bin/bash
# measurement pass: full GPU tests, bench (N=1, with CPU baseline), kernel-trace profile + window anatomy
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/allgpu.log 2>&1
rc=$?; tail -1 gpurun_out/allgpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r01i.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r01i.log | cut -c1-300
bash scripts/prof_only.sh prof_r01i || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --fp8 --no-cpu-baseline --no-vae > gpurun_out/bench_fp8_r01i.log 2>&1; echo fp8 bench rc=$?; tail -1 gpurun_out/bench_fp8_r01i.log | cut -c1-200
