#!/bin/bash
# MX e4m3 path: fp8 kernel tests (incl. the UNet fp8 parity vs the oracle), the MX tile probe, then the fp8 C2 bench
# with the MX producers (default) and with the per-row form (FD_FP8_MX=0).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export FD_PARITY_METRICS=$PWD/gpurun_out/parity_metrics_mx.json
timeout -k 10 500 python -u -m pytest -v --timeout 180 --timeout-method thread tests/test_fp8_gpu.py > gpurun_out/mx_tests.log 2>&1
tail -3 gpurun_out/mx_tests.log
PROBE_MX_TILES=1 timeout -k 10 400 python -u scripts/f8_tiles.py > gpurun_out/f8_tiles_mx.jsonl 2>&1 || exit $?
timeout -k 10 400 python bench.py --fp8 --steps 20 --warmup 3 --no-c3 --no-pipeline --no-cpu-baseline > gpurun_out/bench_fp8_mx.json 2> gpurun_out/bench_fp8_mx.err || exit $?
FD_FP8_MX=0 timeout -k 10 400 python bench.py --fp8 --steps 20 --warmup 3 --no-c3 --no-pipeline --no-cpu-baseline --no-vae > gpurun_out/bench_fp8_row.json 2> gpurun_out/bench_fp8_row.err || exit $?
for f in bench_fp8_mx bench_fp8_row; do python -c "import json;d=json.loads(open('gpurun_out/$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d['roofline_fp8']['achieved'], d['roofline_fp8']['kernel_ms_per_forward'])"; done
