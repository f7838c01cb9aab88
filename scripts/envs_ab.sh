#!/bin/bash
# Interleaved bench-step A/B of env settings: ENVS="A=1,B=2 C=3 ..." (one word per arm, comma-separated vars; "-"
# = defaults), ROUNDS rounds.  Prints ms/step per arm and round.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B="--no-cpu-baseline --no-c3 --no-pipeline --no-roofline --no-vae --steps 40"
for r in $(seq 1 ${ROUNDS:-3}); do
  for arm in $ENVS; do
    e=""; [ "$arm" != "-" ] && e="${arm//,/ }"
    env $e timeout -k 10 200 python bench.py $B > gpurun_out/envs_ab.log 2>&1 || exit $?
    python -c "import json; j=json.loads([l for l in open('gpurun_out/envs_ab.log') if l.startswith('{')][-1]); print('$arm r$r', j['ms_per_step'])"
  done
done
