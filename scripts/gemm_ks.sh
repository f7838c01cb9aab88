#!/bin/bash
# KS (intra-WG split-K) correctness + timing sweep
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FD_GEMM_KS=2 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -p no:cacheprovider -k "gemm or conv or geglu or linear" > gpurun_out/kernels_ks2.log 2>&1
rc=$?; tail -3 gpurun_out/kernels_ks2.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/gemm_ks.jsonl; : > $out
for cfg in 1 0 2; do for ns in 2 4; do for ks in 1 2; do
  FD_GEMM_CFG=$cfg FD_GEMM_NS=$ns FD_GEMM_KS=$ks timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x1280 2048x1280x5120 2048x3840x1280 8192x640x640 8192x1920x640 32768x320x640 >> $out 2>/dev/null || exit $?
done; done; done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/gemm_ks.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    rs=sorted((r for r in rows if r['shape']==shape), key=lambda r:r['us'])
    print(shape, ' | '.join(f"c{r['FD_GEMM_CFG']}n{r['FD_GEMM_NS']}k{r['FD_GEMM_KS']}:{r['us']}" for r in rs[:6]))
PY
