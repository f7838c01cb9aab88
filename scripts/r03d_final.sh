#!/bin/bash
# Final-tree evidence (r03d, after the GroupNorm wide finalize / narrow-conv / MX changes): smoke, the full GPU suite (-v, parity metrics log), the default bench line, and the
# rocprofv3 kernel trace of the bench (step window, GEMM instances, roofline cross-check).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export FD_PARITY_METRICS=$PWD/gpurun_out/r03d_parity_metrics.json
rm -f $FD_PARITY_METRICS
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke.log 2>&1 || { tail -5 gpurun_out/r03d_smoke.log; exit 1; }
tail -2 gpurun_out/r03d_smoke.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03d_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03d_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || exit $?
tail -c 400 gpurun_out/r03d_bench.json
