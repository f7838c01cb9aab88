#!/bin/bash
# r06j: C2 headline / teacher-forced parity, UNet in bf16 (product) and fp16 (the reference's UNet dtype), values
# printed (-s) and recorded
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export FD_PARITY_METRICS=$PWD/gpurun_out/r06j_parity_metrics.json
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_pipeline_gpu.py -k c2_ > gpurun_out/r06j_c2.log 2>&1
rc=$?; grep -E "PSNR|teacher|passed|failed" gpurun_out/r06j_c2.log; exit $rc
