#!/bin/bash
cd "$(dirname "$0")/.."
for cfg in 0 4; do
FD_GEMM_CFG=$cfg timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -p no:cacheprovider -k "gemm or conv or geglu" > gpurun_out/kernels_nl$cfg.log 2>&1
rc=$?; tail -1 gpurun_out/kernels_nl$cfg.log; [ $rc -eq 0 ] || exit $rc
done
out=gpurun_out/gemm_nl.jsonl; : > $out
for cfg in 0 1 4; do for ns in 2 3; do
  FD_GEMM_CFG=$cfg FD_GEMM_NS=$ns timeout -k 5 120 python scripts/gemm_probe.py 2048x10240x1280:geglu 8192x5120x640:geglu 2048x3840x1280 8192x1920x640 32768x1920x640 2048x1280x5120 2048x1280x1280 8192x5120x1280 >> $out 2>/dev/null || exit $?
done; done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/gemm_nl.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    rs=sorted((r for r in rows if r['shape']==shape), key=lambda r:r['us'])
    print(shape, ' | '.join(f"c{r['FD_GEMM_CFG']}n{r['FD_GEMM_NS']}:{r['us']}" for r in rs))
PY
