#!/bin/bash
# Last final-tree check (fp8 default = per-row + MX attention outputs): full GPU suite, then the use_fp8 bench line.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export FD_PARITY_METRICS=$PWD/gpurun_out/r03e_parity_metrics.json
rm -f $FD_PARITY_METRICS
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03e_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03e_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --fp8 --no-c3 --no-pipeline > gpurun_out/r03e_bench_fp8.json 2> gpurun_out/r03e_bench_fp8.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/r03e_bench_fp8.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['roofline_fp8'])"
