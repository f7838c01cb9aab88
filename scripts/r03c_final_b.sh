#!/bin/bash
# Final-tree evidence, part B: kernel trace of the bench, the use_fp8 bench line + its e4m3 PMC traffic pass, C4.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/r02_trace.sh > gpurun_out/r03c_trace.log 2>&1; rc=$?; tail -25 gpurun_out/r03c_trace.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r02_prof.sh unet_fp8 r03c_unet_fp8_pmc > gpurun_out/r03c_unet_fp8_prof.log 2>&1; rc=$?; tail -2 gpurun_out/r03c_unet_fp8_prof.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/traffic_from_pmc.py gpurun_out/r03c_unet_fp8_pmc.json gpurun_out/r03c_gemm_traffic_fp8.json gemm_e4m3 > /dev/null || exit 1
cp gpurun_out/r03c_gemm_traffic_fp8.json profiles/ 2>/dev/null
timeout -k 10 400 python bench.py --fp8 --no-c3 --no-pipeline > gpurun_out/r03c_bench_fp8.json 2> gpurun_out/r03c_bench_fp8.err || exit $?
tail -c 300 gpurun_out/r03c_bench_fp8.json
timeout -k 10 600 python bench.py --workload c4 --steps 20 --warmup 1 > gpurun_out/r03c_bench_c4.json 2> gpurun_out/r03c_bench_c4.err || exit $?
tail -c 300 gpurun_out/r03c_bench_c4.json
