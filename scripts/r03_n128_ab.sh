#!/bin/bash
# 128-channel large-image convs on the 4-wave 128x128 tiles with GroupNorm statistics from their epilogue
# (FD_GEMM8_N128=1, default) vs gemm8 256x128 (=0): tests, then the VAE decode A/B.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_gemm256_gpu.py > gpurun_out/n128_k.log 2>&1
rc=$?; tail -1 gpurun_out/n128_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pipeline_gpu.py -k "vae or tiled or c2_headline" > gpurun_out/n128_p.log 2>&1
rc=$?; tail -1 gpurun_out/n128_p.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/n128.jsonl
for rep in 1 2; do
  AB_TAG=n128off FD_GEMM8_N128=0 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/n128.jsonl || exit $?
  AB_TAG=n128on timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/n128.jsonl || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/n128.jsonl"):
    d = json.loads(l)
    n128 = [t for t in d["top"] if "N=128 " in t[0]]
    print(d.get("AB_TAG"), d["decode_ms_median"], d["decode_ms_min"], d["eager_kind_ms"], n128)
PY
