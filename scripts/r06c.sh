#!/bin/bash
# r06c: full GPU suite on the pruned library (buffer-store sc1 epilogues, ping-pong halo loop, split-K health,
# C4 literal test), smoke, the default bench line, then the one-GPU shard projection
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06c tests smoke bench || exit $?
timeout -k 10 500 python -u scripts/shard_projection.py --out gpurun_out/r06c_shard_projection.json > gpurun_out/r06c_shard.log 2>&1
rc=$?; tail -12 gpurun_out/r06c_shard.log; exit $rc
