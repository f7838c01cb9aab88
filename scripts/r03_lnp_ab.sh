#!/bin/bash
# LN-fold producer at K = 5120 (the 32^2 ff out): 128 x 160 pairwise split (FD_GEMM8_LNP=1) vs 256 x 160 with an
# S-way split (FD_GEMM8_LNP=2, FD_GEMM8_LNP_S); cold weights (PROBE_COPIES), residual + LN partials as in the UNet.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FD_GEMM8_LNP=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ln_fold_gpu.py > gpurun_out/lnp_t.log 2>&1
rc=$?; tail -1 gpurun_out/lnp_t.log; [ $rc -eq 0 ] || exit $rc
export PROBE_LNO=1 PROBE_RES=1 PROBE_COPIES=8
for rep in 1 2; do
  FD_GEMM8_LNP=1 PROBE_TAG=p128s2 timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x5120 || exit $?
  for s in 2 3 4 5; do
    FD_GEMM8_LNP=2 FD_GEMM8_LNP_S=$s PROBE_TAG=p256s$s timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x5120 || exit $?
  done
done
