#!/bin/bash
# Two PMC passes (FETCH_SIZE, WRITE_SIZE do not fit one TCC pass on gfx950), kernel-trace only, no
# runtime/sys trace domains.  Output: gpurun_out/pmc/{fetch,write}/..., parsed by scripts/pmc_parse.py.
cd "$(dirname "$0")/.."
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  d=$R/gpurun_out/pmc/$c
  (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d -o run \
     -- python3 $R/scripts/pmc_traffic.py > $R/gpurun_out/pmc/$c.log 2>&1)
  rc=$?
  echo "$c rc=$rc"; tail -2 $R/gpurun_out/pmc/$c.log
  [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_parse.py
