#!/bin/bash
# ring depth of the 64x160 kernel, warm vs cold weights
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for ns in 4 5; do
FD_GEMM_R4_NS=$ns timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8_gpu.py tests/test_kernels_gpu.py -k "gemm or linear" > gpurun_out/cold_tests.log 2>&1
rc=$?; echo ns=$ns; tail -1 gpurun_out/cold_tests.log; [ $rc -eq 0 ] || exit $rc
done
out=gpurun_out/cold_ab.jsonl; : > $out
S="2048x1280x1280 2048x1280x5120 8192x640x640 2048x3840x1280 2048x10240x1280:geglu"
for c in 1 100; do for ns in 3 4 5; do
  PROBE_COPIES=$c FD_GEMM_R4_NS=$ns timeout -k 5 300 python scripts/gemm_probe.py $S >> $out 2>/dev/null || exit $?
done; FD_GEMM_R4=0 PROBE_COPIES=$c timeout -k 5 300 python scripts/gemm_probe.py $S >> $out 2>/dev/null || exit $?
done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/cold_ab.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    print(f"{shape:24s}", ' | '.join(f"c{r.get('PROBE_COPIES')} {'old' if r.get('FD_GEMM_R4')=='0' else 'ns'+r.get('FD_GEMM_R4_NS','?')}:{r['us']}" for r in rows if r['shape']==shape))
PY
