#!/bin/bash
# Branch-free epilogue activations (rcp SiLU, A&S erf GELU) vs the previous build (probes/ab/lib_oldact.so).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_gemm256_gpu.py > gpurun_out/act_k.log 2>&1
rc=$?; tail -1 gpurun_out/act_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_unet_gpu.py -k "oracle and not fp8" > gpurun_out/act_u.log 2>&1
rc=$?; grep -E "rel_l2|passed|failed" gpurun_out/act_u.log | tail -5; [ $rc -eq 0 ] || exit $rc
S="2048x10240x1280:geglu 8192x5120x640:geglu 2048x1280x1280 conv128x128x320x320"
for rep in 1 2; do
  FD_LIB_PATH=$PWD/probes/ab/lib_oldact.so PROBE_TAG=old timeout -k 5 120 python scripts/gemm_probe.py $S || exit $?
  PROBE_TAG=new timeout -k 5 120 python scripts/gemm_probe.py $S || exit $?
done
for rep in 1 2; do
  AB_TAG=oldact FD_LIB_PATH=$PWD/probes/ab/lib_oldact.so timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_ab2.jsonl || exit $?
  AB_TAG=newact timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_ab2.jsonl || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/vae_ab2.jsonl"):
    d = json.loads(l); print(d.get("AB_TAG"), d["decode_ms_median"], d["decode_ms_min"], d["eager_kind_ms"])
PY
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-c3 --no-pipeline --no-cpu-baseline > gpurun_out/bench_act.json 2> gpurun_out/bench_act.err || exit $?
tail -c 400 gpurun_out/bench_act.json
