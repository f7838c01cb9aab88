#!/bin/bash
# r05ai: the C4 literal reading (1947 tiles) over the full 20-step schedule at the default 25-tile balanced batches
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/c4_literal.py --steps 20 > gpurun_out/r05ai_c4_literal_20.log 2>&1; rc=$?
tail -1 gpurun_out/r05ai_c4_literal_20.log; exit $rc
