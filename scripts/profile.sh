#!/bin/bash
# rocprofv3 kernel-trace stats of the bench (separate from PMC passes, per the MI355X guide).
cd "$(dirname "$0")/.."
R=$(pwd)
NAME=${1:-prof}
export TMPDIR=/tmp
mkdir -p gpurun_out/$NAME
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$NAME -o run \
  -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/$NAME/bench.log 2>&1
rc=$?
echo rc=$rc; tail -3 $R/gpurun_out/$NAME/bench.log
find $R/gpurun_out/$NAME -name "*stats*" | head
exit $rc
