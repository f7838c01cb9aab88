#!/bin/bash
# r05t: final-tree evidence -- smoke, the full GPU suite (parity metrics), the default bench line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05t smoke tests bench || exit $?
