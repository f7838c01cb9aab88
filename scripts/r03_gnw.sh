#!/bin/bash
# Wide GroupNorm finalize: the GroupNorm / conv-statistics kernel tests, then two bench lines (VAE decode ms).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_kernels_gpu.py -k "group_norm or groupnorm" > gpurun_out/gnw_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gnw_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-c3 --no-pipeline --no-cpu-baseline --no-roofline > gpurun_out/gnw_bench$i.json 2> gpurun_out/gnw_bench$i.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/gnw_bench$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['vae_decode_ms'], d.get('vae_kernel_ms'))"
done
