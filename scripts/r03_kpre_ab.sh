#!/bin/bash
# flash d64: K-fragment prefetch under P.V (probes/ab/lib_kpre.so) vs the product build; numerics first.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FD_LIB_PATH=$PWD/probes/ab/lib_kpre.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/kpre_k.log 2>&1
rc=$?; tail -1 gpurun_out/kpre_k.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/base /' || exit $?
  FD_LIB_PATH=$PWD/probes/ab/lib_kpre.so timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/kpre /' || exit $?
done
