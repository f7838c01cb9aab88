#!/bin/bash
# kernel parity tests on the GPU box; output under gpurun_out/
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider > gpurun_out/kernels.log 2>&1
rc=$?
tail -30 gpurun_out/kernels.log
exit $rc
