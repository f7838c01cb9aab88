#!/bin/bash
# r05ac: where the C4 (use_fp8, 13-tile batches) UNet forward spends its time.  rocprofv3 kernel trace of the C4
# leg at 4096^2 output (49 tiles: 13/13/13/10 per step), 2 Euler steps after the 1-step warm-up; per-forward (the last 8 forwards: the timed loop)
# breakdown by kernel instance (scripts/prof_kernel_share.py) and rocprof's kernel stats.
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
D=/tmp/fdprof/c4
rm -rf $D; mkdir -p $D $R/gpurun_out
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run \
   -- python3 $R/bench.py --workload c4 --c4-size 4096 --c3-steps 2 --steps 20 --no-cpu-baseline \
   > $R/gpurun_out/r05ac_prof_c4.log 2>&1)
rc=$?; echo "rocprof rc=$rc"; tail -c 400 $R/gpurun_out/r05ac_prof_c4.log; [ $rc -eq 0 ] || exit $rc
T=$(find $D -name "*kernel_trace.csv" | head -1)
python3 scripts/prof_kernel_share.py $T 45 8 > gpurun_out/r05ac_c4_kernel_share.txt || exit 1
cp $(find $D -name "*kernel_stats.csv" | head -1) gpurun_out/r05ac_c4_kernel_stats.csv
cat gpurun_out/r05ac_c4_kernel_share.txt
