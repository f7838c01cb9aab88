#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider -k "flash" > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
for w in 4 2 8; do FD_FLASH_WAVES=$w timeout -k 5 120 python scripts/attn_probe.py || exit $?; done
