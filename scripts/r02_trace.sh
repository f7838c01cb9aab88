#!/bin/bash
# rocprofv3 kernel trace (+ --stats) of the C2 bench; raw CSVs on the box's /tmp, summaries to gpurun_out:
# per-step window anatomy, per-instance GEMM table, roofline cross-check against the bench line.
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
D=/tmp/fdprof/bench
rm -rf $D; mkdir -p $D $R/gpurun_out
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run \
   -- python3 $R/bench.py --no-cpu-baseline --no-c3 --no-pipeline --steps 20 --warmup 3 > $R/gpurun_out/prof_bench.log 2>&1)
rc=$?; echo "rocprof rc=$rc"; tail -c 300 $R/gpurun_out/prof_bench.log; [ $rc -eq 0 ] || exit $rc
T=$(find $D -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_window.py $T 3 > gpurun_out/prof_window.txt || exit 1
python3 scripts/roofline_check.py $T gpurun_out/prof_bench.log 3 > gpurun_out/prof_roofline_check.json || exit 1
python3 scripts/prof_gemm_breakdown.py $T 3 > gpurun_out/prof_gemm_instances.txt 2>&1 || true
cp $(find $D -name "*kernel_stats.csv" | head -1) gpurun_out/prof_kernel_stats.csv
head -20 gpurun_out/prof_window.txt; cat gpurun_out/prof_roofline_check.json
