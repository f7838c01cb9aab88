#!/bin/bash
# r05y: C4 in its literal reading, the full 20-step schedule (1947 TLC tiles, 30720x17280 output)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/c4_literal.py --steps 20 2>&1 | tee gpurun_out/r05y_c4_literal_20.log
