#!/bin/bash
# In-session A/B on one box: gemm256 (old vs ping-pong), GroupNorm apply (v1 vs v2), flash softmax fma (packed vs scalar).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or flash or group_norm" > gpurun_out/ab1_tests.log 2>&1
rc=$?; tail -1 gpurun_out/ab1_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  FD_LIB_PATH=$PWD/build_ab/libA.so timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/old /' || exit $?
  timeout -k 5 120 python scripts/attn_probe.py | sed 's/^/new /' || exit $?
done
for rep in 1 2; do
  AB_TAG=g256old FD_LIB_PATH=$PWD/build_ab/libG.so timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_ab.jsonl || exit $?
  AB_TAG=new timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_ab.jsonl || exit $?
  AB_TAG=gnv1 FD_GN_APPLY_V=1 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_ab.jsonl || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/vae_ab.jsonl"):
    d = json.loads(l); print(d.get("AB_TAG"), d["decode_ms_median"], d["decode_ms_min"], d["eager_kind_ms"])
PY
