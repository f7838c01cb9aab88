#!/bin/bash
# e4m3 eight-wave kernel: fp8 kernel tests, the tile A/B probe, then the fp8 C2 bench line.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fp8_gpu.py > gpurun_out/f8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/f8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/f8_tiles.py > gpurun_out/f8_tiles.jsonl 2>&1 || exit $?
cat gpurun_out/f8_tiles.jsonl
timeout -k 10 400 python bench.py --fp8 --steps 20 --warmup 3 --no-c3 --no-pipeline --no-cpu-baseline > gpurun_out/bench_fp8.json 2> gpurun_out/bench_fp8.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/bench_fp8.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('roofline_fp8', d.get('roofline')))"
