#!/bin/bash
# pairwise split-K (S = 2): correctness under each forcing, then per-shape A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for env in "FD_GEMM_P128=1" "FD_GEMM8_S=2"; do
  env $env timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8_gpu.py tests/test_kernels_gpu.py -k "gemm or conv or linear or geglu" > gpurun_out/pair_tests.log 2>&1
  rc=$?; echo "$env"; tail -3 gpurun_out/pair_tests.log; [ $rc -eq 0 ] || exit $rc
done
out=gpurun_out/pair_ab.jsonl; : > $out
S="2048x1280x1280 2048x1280x5120 2048x1280x2560 2048x3840x1280 2048x10240x1280:geglu 8192x640x640 8192x640x2560 conv32x32x1280x1280"
timeout -k 5 120 python scripts/gemm_probe.py $S >> $out 2>/dev/null || exit $?
FD_GEMM_P128=1 timeout -k 5 120 python scripts/gemm_probe.py $S >> $out 2>/dev/null || exit $?
FD_GEMM8_S=2 timeout -k 5 120 python scripts/gemm_probe.py $S >> $out 2>/dev/null || exit $?
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/pair_ab.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    print(f"{shape:26s}", ' | '.join(f"{'P128' if r.get('FD_GEMM_P128') else ('S2' if r.get('FD_GEMM8_S') else 'base')}:{r['us']}" for r in rows if r['shape']==shape))
PY
