#!/bin/bash
# Round-4 start: the new parity cases (odd-size UNet, reference-forward golden, 8-image C5, batched-call forwarding),
# then the C2 bench line and its kernel trace on the current tree.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_unet_gpu.py \
  tests/test_configs_gpu.py -k "forward_matches or c5_images or forwards_embeddings" > gpurun_out/r04a_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r04a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline --no-c3 --no-pipeline > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit $?
tail -c 600 gpurun_out/r04a_bench.json
bash scripts/r02_trace.sh > gpurun_out/r04a_trace.log 2>&1; rc=$?; tail -25 gpurun_out/r04a_trace.log; exit $rc
