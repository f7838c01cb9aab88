#!/bin/bash
# Flash attention d64 variants on one box: compile-time (probes/ab/lib_*.so) and launch-shape knobs (env).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FD_LIB_PATH=$PWD/probes/ab/lib_qpre.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/qpre_k.log 2>&1
rc=$?; tail -1 gpurun_out/qpre_k.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
FD_LIB_PATH=$PWD/probes/ab/lib_qpre.so timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_unet_gpu.py -k "oracle and not fp8" > gpurun_out/qpre_u.log 2>&1
rc=$?; grep -E "rel_l2|passed|failed" gpurun_out/qpre_u.log | tail -5; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
  timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/base /' || exit $?
  for v in nb2 nb4 tr0 qpre; do
    FD_LIB_PATH=$PWD/probes/ab/lib_$v.so timeout -k 5 120 python scripts/attn_probe.py | sed "s/^/$v /" || exit $?
  done
  FD_FLASH_WAVES=8 timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/w8 /' || exit $?
  FD_FLASH_WAVES=2 timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/w2 /' || exit $?
  FD_FLASH_QPW=32 timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/q32 /' || exit $?
done
