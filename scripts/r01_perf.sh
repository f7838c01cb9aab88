#!/bin/bash
# kernel parity, per-shape tables (flash XCD remap off/on), kernel-trace profile of the bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -p no:cacheprovider > gpurun_out/kernels.log 2>&1
rc=$?; tail -2 gpurun_out/kernels.log; [ $rc -eq 0 ] || exit $rc
FD_FLASH_SWZ=0 timeout -k 10 300 python scripts/shape_table.py > gpurun_out/shape_swz0.log 2>&1 || exit $?
timeout -k 10 300 python scripts/shape_table.py > gpurun_out/shape_swz1.log 2>&1 || exit $?
grep flash gpurun_out/shape_swz0.log | head -4; grep flash gpurun_out/shape_swz1.log | head -4
bash scripts/profile.sh prof_r01
