#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8_gpu.py tests/test_ln_fold_gpu.py tests/test_kernels_gpu.py -k "geglu or gemm or consumer" > gpurun_out/w160_tests.log 2>&1
rc=$?; tail -1 gpurun_out/w160_tests.log; [ $rc -eq 0 ] || exit $rc
for w in 0 1; do
FD_GEMM8_W160=$w timeout -k 5 120 python scripts/gemm_probe.py 2048x10240x1280:geglu 8192x5120x640:geglu | sed "s/^/w160=$w /"
FD_GEMM8_W160=$w timeout -k 5 120 python scripts/lnf_probe.py | sed "s/^/w160=$w /"
done
bash scripts/env_ab.sh FD_GEMM8_W160=0 > gpurun_out/env_ab.log 2>&1; cat gpurun_out/env_ab.log
