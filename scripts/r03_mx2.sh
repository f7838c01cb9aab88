#!/bin/bash
# fp8 C2 step A/B, three forms on one box: MX producers with the GEGLU in bf16 + MX quantization (default), MX GEGLU
# epilogue (FD_FP8_MX_GEGLU=1), per-row e4m3 (FD_FP8_MX=0).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_fp8_gpu.py -k "layer_norm_mx or unet" > gpurun_out/mx2_tests.log 2>&1
tail -2 gpurun_out/mx2_tests.log
for rep in 1; do
for v in "mx:" "mxg:FD_FP8_MX_GEGLU=1" "row:FD_FP8_MX=0"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --fp8 --steps 40 --warmup 3 --no-c3 --no-pipeline --no-cpu-baseline --no-vae --no-roofline > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1]);print('$tag rep$rep', d['ms_per_step'])"
done
done
