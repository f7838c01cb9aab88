#!/bin/bash
# rocprofv3 kernel trace (+ --stats) of the C2 bench; raw CSVs on the box's /tmp, summaries to gpurun_out/<tag>_*:
# per-step window anatomy, per-instance GEMM table, roofline cross-check against the bench line, kernel stats.
# Usage: scripts/trace.sh <tag> [extra bench.py args]
cd "$(dirname "$0")/.."
R=$(pwd)
TAG=${1:-trace}; shift
export TMPDIR=/tmp
D=/tmp/fdprof/bench
rm -rf $D; mkdir -p $D $R/gpurun_out
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run \
   -- python3 $R/bench.py --no-cpu-baseline --no-c3 --no-pipeline --steps 20 --warmup 3 "$@" > $R/gpurun_out/${TAG}_prof_bench.log 2>&1)
rc=$?; echo "rocprof rc=$rc"; tail -c 300 $R/gpurun_out/${TAG}_prof_bench.log; [ $rc -eq 0 ] || exit $rc
T=$(find $D -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_window.py $T 3 > gpurun_out/${TAG}_step_window.txt || exit 1
python3 scripts/roofline_check.py $T gpurun_out/${TAG}_prof_bench.log 3 > gpurun_out/${TAG}_roofline_check.json || exit 1
python3 scripts/prof_gemm_breakdown.py $T 3 > gpurun_out/${TAG}_gemm_instances.txt 2>&1 || true
python3 scripts/prof_positions.py $T 3 > gpurun_out/${TAG}_positions.txt 2>&1 || true
cp $(find $D -name "*kernel_stats.csv" | head -1) gpurun_out/${TAG}_kernel_stats.csv
gzip -c $T > gpurun_out/${TAG}_kernel_trace.csv.gz  # the raw trace, for off-box analysis (scripts/prof_*.py read .gz)
head -20 gpurun_out/${TAG}_step_window.txt; cat gpurun_out/${TAG}_roofline_check.json
