#!/bin/bash
# Mid-K launches with < 192 tiles of 256 rows (the 4-wave kernel's today): forced gemm8 split-K (S = 2, 3)
# against the default, at C2 (one tile) and at C3's batching (13 tiles per launch), cold weights.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/ksplit.jsonl; : > $out
export PROBE_COPIES=24
c2="2048x1280x5120 conv64x64x640x640 conv32x32x1280x1280 conv32x32x640x1280"
run() { timeout -k 5 150 python scripts/gemm_probe.py "$@" >> $out 2>>gpurun_out/ksplit.err; }
for s in 0 2 3; do
  unset FD_GEMM8_S; [ $s -gt 0 ] && export FD_GEMM8_S=$s
  run $c2 || exit $?
  PROBE_GROUPS=13 PROBE_NIMG=26 run 26624x1280x5120 conv64x64x640x640 || exit $?
done
python - <<'PY'
import json
for l in open('gpurun_out/ksplit.jsonl'):
    r = json.loads(l)
    k = {a: b for a, b in r.items() if a not in ('shape', 'us', 'tflops', 'PROBE_COPIES')}
    print(f"{r['shape']:>22} {r['us']:9.2f} us {r['tflops']:7.1f} TF  {k}")
PY
