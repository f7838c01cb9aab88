#!/bin/bash
# 128x160 S=1 for the large-M GEMMs / convs: correctness, then A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FD_GEMM_B4=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm8_gpu.py tests/test_kernels_gpu.py -k "gemm or conv or linear or geglu" > gpurun_out/b4_tests.log 2>&1
rc=$?; tail -1 gpurun_out/b4_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/b4_ab.jsonl; : > $out
S="conv128x128x320x320 conv64x64x640x640 conv128x128x640x320 conv64x64x1280x640 8192x640x640 8192x640x2560 32768x320x640 32768x640x1280 32768x1920x640 8192x1920x640"
for b in 0 1; do
  FD_GEMM_B4=$b timeout -k 5 300 python scripts/gemm_probe.py $S >> $out 2>/dev/null || exit $?
done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/b4_ab.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    print(f"{shape:24s}", ' | '.join(f"b4={r.get('FD_GEMM_B4')}:{r['us']}" for r in rows if r['shape']==shape))
PY
