#!/bin/bash
# Flash tail-tile key-block skip: tests, then interleaved probes / bench steps against the previous attention build
# (faithdiff-dev_amd/fdhip/diag/lib_oldattn.so).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OLD=$(pwd)/faithdiff-dev_amd/fdhip/diag/lib_oldattn.so
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_clip_gpu.py > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -2 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  FD_FLASH_TAG=old FD_LIB_PATH=$OLD timeout -k 10 120 python scripts/attn_probe.py 2x20x1024x77 2x10x4096x77 2x20x1024x1024 1x20x77x77 2>/dev/null || exit $?
  FD_FLASH_TAG=new timeout -k 10 120 python scripts/attn_probe.py 2x20x1024x77 2x10x4096x77 2x20x1024x1024 1x20x77x77 2>/dev/null || exit $?
done
B="--no-cpu-baseline --no-c3 --no-pipeline --no-roofline --no-vae --steps 40"
for r in 1 2 3; do
  FD_LIB_PATH=$OLD timeout -k 10 200 python bench.py $B > gpurun_out/tail_b.log 2>&1 || exit $?
  python -c "import json; j=json.loads([l for l in open('gpurun_out/tail_b.log') if l.startswith('{')][-1]); print('old r$r', j['ms_per_step'])"
  timeout -k 10 200 python bench.py $B > gpurun_out/tail_b.log 2>&1 || exit $?
  python -c "import json; j=json.loads([l for l in open('gpurun_out/tail_b.log') if l.startswith('{')][-1]); print('new r$r', j['ms_per_step'])"
done
