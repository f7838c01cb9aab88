#!/bin/bash
# C3 (4096^2, 49 tiles) at several TLC tile batches (FD_TILE_BATCH), one rank
cd "$(dirname "$0")/.."
for tb in ${TBS:-4 7 13 25}; do
  FD_TILE_BATCH=$tb timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --no-vae --no-pipeline \
    --no-roofline > gpurun_out/tb_$tb.log 2>&1 || exit $?
  echo "tb=$tb $(grep '^{"metric"' gpurun_out/tb_$tb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d.get("c3",d); print(d["value"], c.get("s_per_image"), c.get("step_ms_median"))')"
done
