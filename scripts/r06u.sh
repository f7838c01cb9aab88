#!/bin/bash
# r06u: the committed final tree once more -- the whole -m gpu suite and smoke
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06u tests smoke
