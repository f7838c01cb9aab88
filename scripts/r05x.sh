#!/bin/bash
# r05x: C4 in its literal reading (7680x4320 x4 -> 30720x17280, 1947 TLC tiles), one denoise step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/c4_literal.py --steps 1 2>&1 | tee gpurun_out/r05x_c4_literal.log
