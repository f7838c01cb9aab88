#!/bin/bash
# gemm8 conv shapes (graph-timed): the VAE's 128-channel convs at 1024^2 and the UNet's convs
cd "$(dirname "$0")/.."
SH="conv512x1024x128x128 conv32x32x1280x1280 conv64x64x640x640 conv128x128x320x320 conv256x512x256x256"
out=gpurun_out/g8_probe.jsonl; : > $out
FD_GEMM256=0 timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
cat $out
