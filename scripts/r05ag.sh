#!/bin/bash
# r05ag: final-tree evidence after the tile-batch defaults -- smoke and the full GPU suite (call 1, "tests"), then the
# default bench line and the C4 bench line (call 2, "bench")
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
case $1 in
  tests) bash scripts/run.sh r05ag smoke tests || exit $? ;;
  bench) bash scripts/run.sh r05ag bench && \
         timeout -k 10 400 python bench.py --workload c4 --no-cpu-baseline > gpurun_out/r05ag_bench_c4.json 2> gpurun_out/r05ag_bench_c4.err && \
         tail -c 600 gpurun_out/r05ag_bench_c4.json ;;
esac
