#!/bin/bash
# Narrow-N conv_out: kernel tests, the VAE / pipeline parity tests, then the VAE decode A/B (FD_VAE_NARROW=0 / 1).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export FD_PARITY_METRICS=$PWD/gpurun_out/parity_metrics_narrow.json
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_kernels_gpu.py -k "narrow" > gpurun_out/narrow_tests.log 2>&1
rc=$?; tail -2 gpurun_out/narrow_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py > gpurun_out/narrow_pipe_tests.log 2>&1
rc=$?; tail -2 gpurun_out/narrow_pipe_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 1 0; do
FD_VAE_NARROW=$v timeout -k 10 300 python bench.py --no-c3 --no-pipeline --no-cpu-baseline --no-roofline --steps 5 > gpurun_out/narrow_b$v.json 2> gpurun_out/narrow_b$v.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/narrow_b$v.json').read().strip().splitlines()[-1]);print('narrow=$v', d['vae_decode_ms'], d.get('vae_kernel_ms'))"
done; done
