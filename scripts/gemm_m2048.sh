#!/bin/bash
# M=2048 projection family: load-only (mode 1) / compute-only (mode 2) / full, per tile config and ring depth
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/gemm_m2048.jsonl; : > $out
for cfg in 1 0 2 3; do for ns in 2 3 4; do for mode in 0 1 2; do
  FD_GEMM8=0 FD_GEMM_CFG=$cfg FD_GEMM_NS=$ns FD_GEMM_MODE=$mode timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x1280 2048x1280x5120 >> $out 2>/dev/null || exit $?
done; done; done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/gemm_m2048.jsonl')]
for r in rows:
    print(r['shape'], 'cfg', r.get('FD_GEMM_CFG'), 'ns', r.get('FD_GEMM_NS'), 'mode', r.get('FD_GEMM_MODE'), r['us'])
PY
