#!/bin/bash
# A/B: in-tree library vs build_ab/libB.so, interleaved rounds in one call
cd "$(dirname "$0")/.."
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider -k "flash" > gpurun_out/attn_tests.log 2>&1
rc=$?; tail -1 gpurun_out/attn_tests.log; [ $rc -eq 0 ] || exit $rc
FD_LIB_PATH=build_ab/libB.so timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider -k "flash" > gpurun_out/attn_testsB.log 2>&1
rc=$?; tail -1 gpurun_out/attn_testsB.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  FD_FLASH_VARIANT=A timeout -k 5 120 python scripts/attn_probe.py || exit $?
  FD_FLASH_VARIANT=B FD_LIB_PATH=build_ab/libB.so timeout -k 5 120 python scripts/attn_probe.py || exit $?
done
