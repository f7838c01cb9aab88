#!/bin/bash
# r06d: in-context vs family-graph losses: the C2 forward and its kernel-family graphs under a
# kernel trace with the side-stream clock sampler running (per-launch shader clock), then one TCC_HIT / TCC_MISS pass;
# the trace / counter CSVs come back gzipped for scripts/incontext_report.py
cd "$(dirname "$0")/.."
R=$(pwd)
TAG=${1:-r06d}
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/fdprof/incontext
rm -rf $D; mkdir -p $D
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o run \
   -- python3 $R/scripts/incontext_probe.py --tag ${TAG} > $R/gpurun_out/${TAG}_trace.log 2>&1) || { tail -5 gpurun_out/${TAG}_trace.log; exit 1; }
grep -E "^(idle|forward|proj|flash|gemm) " gpurun_out/${TAG}_trace.log
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $D/pmc -o run \
   -- python3 $R/scripts/incontext_probe.py --tag ${TAG}_pmc --no-clock --reps 2 > $R/gpurun_out/${TAG}_pmc.log 2>&1) || { tail -5 gpurun_out/${TAG}_pmc.log; exit 1; }
T=$(find $D/trace -name "*kernel_trace.csv" | head -1)
P=$(find $D/pmc -name "*counter_collection.csv" | head -1)
gzip -c $T > gpurun_out/${TAG}_incontext_trace.csv.gz
gzip -c $P > gpurun_out/${TAG}_tcc.csv.gz
python3 scripts/incontext_report.py $T --samples gpurun_out/${TAG}_samples.npz --pmc $P > gpurun_out/${TAG}_incontext.json; rc=$?
cat gpurun_out/${TAG}_incontext.json | head -80; exit $rc
