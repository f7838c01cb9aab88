#!/bin/bash
# Fixed vs per-K-step cost of the 64x160 gemm_kernel at M = 2048, N = 1280 (the 32^2-level projections):
# graph-timed launches (scripts/gemm_probe.py) at K = 640..10240, full kernel / loads only / LDS + MFMA only,
# plain and with the residual + LayerNorm-partials epilogue of the product's residual-stream GEMMs.
cd "$(dirname "$0")/.."
out=gpurun_out/gemm_k_sweep.jsonl; : > $out
for mode in 0 1 2; do for epi in 0 1; do
  FD_GEMM8=0 FD_GEMM_CFG=1 FD_GEMM_MODE=$mode PROBE_RES=$epi PROBE_LNO=$epi PROBE_TAG=epi$epi \
    timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x640 2048x1280x1280 2048x1280x2560 2048x1280x5120 \
    2048x1280x10240 >> $out 2>/dev/null || exit $?
done; done
cat $out
