#!/bin/bash
# rocprofv3 kernel trace (+ --stats) of the use_fp8 C2 bench on the final tree: per-step window anatomy.
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
D=/tmp/fdprof/bench_fp8
rm -rf $D; mkdir -p $D $R/gpurun_out
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run \
   -- python3 $R/bench.py --fp8 --no-cpu-baseline --no-c3 --no-pipeline --no-vae --no-roofline --steps 20 --warmup 3 > $R/gpurun_out/prof_bench_fp8.log 2>&1)
rc=$?; echo "rocprof rc=$rc"; tail -c 200 $R/gpurun_out/prof_bench_fp8.log; [ $rc -eq 0 ] || exit $rc
T=$(find $D -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_window.py $T 3 > gpurun_out/r03e_fp8_step_window.txt || exit 1
cp $(find $D -name "*kernel_stats.csv" | head -1) gpurun_out/r03e_fp8_kernel_stats.csv
head -16 gpurun_out/r03e_fp8_step_window.txt
