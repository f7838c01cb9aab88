#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or flash" > gpurun_out/attn_t.log 2>&1
rc=$?; tail -1 gpurun_out/attn_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_clip_gpu.py > gpurun_out/attn_t2.log 2>&1
rc=$?; tail -1 gpurun_out/attn_t2.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
FD_LIB_PATH=$PWD/build_ab/libA.so timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/old /' || exit $?
timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/new /' || exit $?
done
