#!/bin/bash
# kernels + gemm8 + unet parity, then one bench line (no CPU baseline)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_unet_gpu.py tests/test_clip_gpu.py > gpurun_out/qc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/qc_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-vae --steps 30 > gpurun_out/qc_bench.log 2>&1 || exit $?
tail -1 gpurun_out/qc_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["attention"] if "attention" in d else "")'
done
