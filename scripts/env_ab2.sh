#!/bin/bash
# interleaved bench A/B of environment knobs on one box: scripts/env_ab2.sh "ENV=.. ENV2=.." "..." ...
cd "$(dirname "$0")/.."
for r in 1 2; do
  for cfg in "" "$@"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 --no-pipeline --no-vae --no-roofline \
      > gpurun_out/envab.log 2>&1 || exit $?
    echo "[$cfg] $(grep '^{"metric"' gpurun_out/envab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done
done
