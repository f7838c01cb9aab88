#!/bin/bash
# GroupNorm apply: 4 vs 8 16-B vectors in flight per thread (FD_GN_APPLY_U), interleaved: C2 step + VAE decode.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B="--no-cpu-baseline --no-c3 --no-pipeline --no-roofline --steps 30"
for r in 1 2; do
  for u in 4 8; do
    FD_GN_APPLY_U=$u timeout -k 10 250 python bench.py $B > gpurun_out/gnu_${u}_$r.log 2>&1 || exit $?
    python -c "import json; j=json.loads([l for l in open('gpurun_out/gnu_${u}_$r.log') if l.startswith('{')][-1]); print('U=$u r$r', j['ms_per_step'], j.get('vae_decode_ms'), j.get('vae_norm', {}).get('achieved'), j.get('vae_norm', {}).get('ms'))"
  done
done
