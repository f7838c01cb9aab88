#!/bin/bash
# M = 2048, N = 1280 projections (the 32^2 level at C2, 196 launches per step): the 4-wave 64x160 kernel
# (default) against gemm8 with in-launch split-K (256x128 tiles, S = 2..4) and the 128x160 pairwise form,
# warm (one weight copy) and cold (weights cycled past the Infinity Cache, as inside a UNet forward).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/m2048_split.jsonl; : > $out
run() { timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x5120 2048x1280x1280 >> $out 2>>gpurun_out/m2048_split.err; }
for copies in 1 24; do
  export PROBE_COPIES=$copies
  run || exit $?
  for s in 2 3 4 5; do FD_GEMM8_S=$s run || exit $?; done
  FD_GEMM_R4=1 FD_GEMM_P128=1 run || exit $?
  FD_GEMM_R4=1 run || exit $?
done
python - <<'PY'
import json
for l in open('gpurun_out/m2048_split.jsonl'):
    r = json.loads(l)
    k = {a: b for a, b in r.items() if a not in ('shape', 'us', 'tflops')}
    print(f"{r['shape']:>16} {r['us']:8.2f} us {r['tflops']:7.1f} TF  {k}")
PY
