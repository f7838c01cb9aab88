#!/bin/bash
# A/B of gemm8's ping-pong main loop (FD_GEMM_PP=1, default) against the single-group loop (FD_GEMM_PP=0) on the
# UNet's eight-wave shapes, graph-timed by scripts/gemm_probe.py, interleaved rounds in separate processes.
cd "$(dirname "$0")/.."
out=gpurun_out/pp_ab.jsonl; : > $out
SH="2048x10240x1280:geglu 2048x3840x1280 8192x5120x640:geglu 8192x1920x640 8192x640x2560 conv64x64x640x640 conv32x32x1280x1280 conv128x128x320x320"
for r in 1 2; do for pp in 0 1; do
  FD_GEMM_PP=$pp PROBE_TAG=r$r timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
done; done
cat $out
