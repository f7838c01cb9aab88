#!/bin/bash
# r06p: record the C2 forward's GEMM-family launches (8-XCD traffic floor, scripts/gemm_traffic_floor.py) and run
# C5 through all 50 steps of its schedule in the GPU suite
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_traffic_floor.py --record gpurun_out/r06p_gemm_launches.json \
  --traffic profiles/r06l_gemm_traffic.json --out gpurun_out/r06p_gemm_traffic_floor.json > gpurun_out/r06p_floor.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread \
  "tests/test_configs_gpu.py::test_c5_full_50_step_schedule_8_images" > gpurun_out/r06p_c5_full.log 2>&1
rc=$?; tail -3 gpurun_out/r06p_floor.log; tail -3 gpurun_out/r06p_c5_full.log; exit $rc
