#!/bin/bash
# r06q: final-tree evidence after the concat + GroupNorm-statistics fusion: the whole -m gpu suite, smoke, the default
# bench line (the driver's command), and the C2 kernel trace
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06q tests smoke bench trace
