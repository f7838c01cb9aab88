#!/bin/bash
# 64x160 one-wave-per-SIMD kernel: correctness, then A/B against the 4-wave kernel per shape
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8_gpu.py tests/test_kernels_gpu.py -k "gemm or conv or linear or geglu" > gpurun_out/r4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_tests.log; [ $rc -eq 0 ] || exit $rc
FD_GEMM_R4=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8_gpu.py tests/test_kernels_gpu.py -k "gemm or conv or linear or geglu" > gpurun_out/r4_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/r4_tests2.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/r4_ab.jsonl; : > $out
for r4 in 0 1 2; do
  FD_GEMM_R4=$r4 timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x1280 2048x1280x5120 2048x1280x2560 8192x640x640 8192x640x2560 32768x320x640 32768x640x1280 conv64x64x640x640 conv128x128x320x320 conv32x32x1280x1280 >> $out 2>/dev/null || exit $?
done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/r4_ab.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    print(shape, ' | '.join(f"r4={r.get('FD_GEMM_R4')}:{r['us']}" for r in rows if r['shape']==shape))
PY
