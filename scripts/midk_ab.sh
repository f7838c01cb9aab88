#!/bin/bash
# A/B of a planner switch (VAR=0 = off; default FD_GEMM8_MIDK, the mid-K split rule) in the bench step,
# interleaved on one box; then C3.  TESTS: the GPU test files run first.
cd "$(dirname "$0")/.."
VAR=${VAR:-FD_GEMM8_MIDK}
TESTS=${TESTS:-"tests/test_gemm8_gpu.py tests/test_unet_gpu.py"}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > gpurun_out/midk_tests.log 2>&1
rc=$?; tail -2 gpurun_out/midk_tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-c3 --no-pipeline --no-roofline --no-vae --steps 40"
for r in 1 2 3; do
  env $VAR=0 timeout -k 10 200 python bench.py $B > gpurun_out/midk_off$r.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py $B > gpurun_out/midk_on$r.log 2>&1 || exit $?
done
for n in off1 on1 off2 on2 off3 on3; do
  python -c "import json,sys; j=json.loads([l for l in open('gpurun_out/midk_$n.log') if l.startswith('{')][-1]); print('$n', j['ms_per_step'])"
done
env $VAR=0 timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/midk_c3_off.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/midk_c3_on.log 2>&1 || exit $?
for n in c3_off c3_on; do
  python -c "import json,sys; j=json.loads([l for l in open('gpurun_out/midk_$n.log') if l.startswith('{')][-1]); print('$n', j['value'], j['ms_per_step'])"
done
