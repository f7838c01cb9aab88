#!/bin/bash
# r06a: halo conv ping-pong K loop -- halo GPU tests (incl. PP vs one-barrier bitwise), split-K timeout path, the
# timestep-row test; per-shape A/B; step + VAE A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06a "tfile=tests/test_conv_halo_gpu.py" "tfile=tests/test_splitk_health_gpu.py" \
  "tfile=tests/test_kernels_gpu.py:scale_input" smoke || exit $?
for pp in 1 0; do
  FD_CONV_HALO_PP=$pp timeout -k 10 300 python -u probes/conv_ab.py > gpurun_out/r06a_conv_ab_pp$pp.jsonl 2>&1 || exit $?
done
bash scripts/run.sh r06a "abv=2;FD_CONV_HALO_PP=1;FD_CONV_HALO_PP=0" || exit $?
