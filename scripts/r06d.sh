#!/bin/bash
# r06d: in-context vs family-graph losses: the shader clock per phase (side-stream sampler),
# a kernel trace of the same phases, one TCC_HIT / TCC_MISS pass; then scripts/incontext_report.py
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/fdprof/incontext
rm -rf $D; mkdir -p $D
timeout -k 10 300 python -u scripts/incontext_probe.py --tag r06d > gpurun_out/r06d_clock.log 2>&1 || { tail -20 gpurun_out/r06d_clock.log; exit 1; }
tail -6 gpurun_out/r06d_clock.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run \
   -- python3 $R/scripts/incontext_probe.py --tag r06d_tr --no-clock > $R/gpurun_out/r06d_trace.log 2>&1) || { tail -5 gpurun_out/r06d_trace.log; exit 1; }
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $D/pmc -o run \
   -- python3 $R/scripts/incontext_probe.py --tag r06d_pmc --no-clock --reps 2 > $R/gpurun_out/r06d_pmc.log 2>&1) || { tail -5 gpurun_out/r06d_pmc.log; exit 1; }
T=$(find $D/trace -name "*kernel_trace.csv" | head -1)
P=$(find $D/pmc -name "*counter_collection.csv" | head -1)
python3 scripts/incontext_report.py $T $P > gpurun_out/r06d_incontext.json; rc=$?
cat gpurun_out/r06d_incontext.json; exit $rc
