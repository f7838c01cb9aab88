#!/bin/bash
# gemm8 parity, then graph-timed old (FD_GEMM8=0) vs new kernel, and split-count sweep on the C2 shapes.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gemm8_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -p no:cacheprovider -k "gemm or conv" > gpurun_out/gemm8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gemm8_tests.log; [ $rc -eq 0 ] || exit $rc
out=gpurun_out/gemm8_sweep.jsonl; : > $out
SH="2048x1280x1280 2048x1280x5120 2048x3840x1280 2048x10240x1280:geglu conv32x32x1280x1280 8192x640x640 8192x5120x640:geglu conv64x64x640x640 conv128x128x320x320 32768x1920x640"
FD_GEMM8=0 timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>gpurun_out/gemm8_sweep.err || exit $?
timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>>gpurun_out/gemm8_sweep.err || exit $?
for s in 1 2 3 4 6 8; do
  FD_GEMM8_S=$s timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>>gpurun_out/gemm8_sweep.err || exit $?
done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/gemm8_sweep.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    rs=[r for r in rows if r['shape']==shape]
    old=[r['us'] for r in rs if r.get('FD_GEMM8')=='0']
    new=[r['us'] for r in rs if 'FD_GEMM8' not in r and 'FD_GEMM8_S' not in r]
    ss=' '.join(f"S{r['FD_GEMM8_S']}:{r['us']}" for r in rs if 'FD_GEMM8_S' in r)
    print(f"{shape:28s} old {old} new {new} | {ss}")
PY
