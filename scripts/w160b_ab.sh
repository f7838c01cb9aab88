#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in 1 3; do
FD_GEMM8_W160=$w timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm8_gpu.py tests/test_kernels_gpu.py tests/test_ln_fold_gpu.py > gpurun_out/w160_tests.log 2>&1
rc=$?; echo "w160=$w $(tail -1 gpurun_out/w160_tests.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_unet_gpu.py > gpurun_out/w160_unet.log 2>&1
rc=$?; echo "unet $(tail -1 gpurun_out/w160_unet.log)"; [ $rc -eq 0 ] || exit $rc
for w in 0 1 3; do
FD_GEMM8_W160=$w timeout -k 5 200 python scripts/gemm_probe.py conv32x32x1280x1280 conv64x64x1920x640 conv128x128x320x320 conv128x128x640x320 32768x640x1280 | sed "s/^/w160=$w /"
done
bash scripts/env_ab.sh FD_GEMM8_W160=0 FD_GEMM8_W160=3 > gpurun_out/env_ab.log 2>&1; cat gpurun_out/env_ab.log
