#!/bin/bash
# flash d64: half of the next tile's K fragments read under P.V, 3-wave occupancy target (probes/ab/lib_k2w3.so)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FD_LIB_PATH=$PWD/probes/ab/lib_k2w3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/kpre2_k.log 2>&1
rc=$?; tail -1 gpurun_out/kpre2_k.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/base /' || exit $?
  FD_LIB_PATH=$PWD/probes/ab/lib_k2w3.so timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/k2w3 /' || exit $?
done
