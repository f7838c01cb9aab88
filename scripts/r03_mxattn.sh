#!/bin/bash
# fp8: MX only for the attention outputs (FD_FP8_MX_ATTN=1) vs per-row everywhere (default) vs MX everywhere
# (FD_FP8_MX=1): fp8 parity tests, then the C2 step A/B alternated on one box.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export FD_PARITY_METRICS=$PWD/gpurun_out/parity_metrics_mxattn.json
FD_FP8_MX_ATTN=1 timeout -k 10 400 python -u -m pytest -q --timeout 180 --timeout-method thread tests/test_fp8_gpu.py -k "unet or pipeline" > gpurun_out/mxattn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/mxattn_tests.log; [ $rc -eq 0 ] || exit $rc
grep "unet fp8\|PSNR" gpurun_out/mxattn_tests.log | head
for rep in 1 2; do
for v in "hyb:FD_FP8_MX_ATTN=1" "row:" "mx:FD_FP8_MX=1"; do
  tag=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python bench.py --fp8 --steps 40 --warmup 3 --no-c3 --no-pipeline --no-cpu-baseline --no-vae --no-roofline > gpurun_out/ma_$tag.json 2> gpurun_out/ma_$tag.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/ma_$tag.json').read().strip().splitlines()[-1]);print('$tag rep$rep', d['ms_per_step'])"
done
done
