#!/bin/bash
# r06k: final-tree GPU suite, smoke, the default bench line, the fp16-UNet C2 line, the C4 line (use_fp8, e4m3 MFMA)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06k tests smoke bench "bench=--unet-fp16,--no-c3,--no-pipeline,--no-cpu-baseline" || exit $?
timeout -k 10 400 python bench.py --workload c4 --steps 20 --no-cpu-baseline > gpurun_out/r06k_bench_c4.json 2> gpurun_out/r06k_bench_c4.err
rc=$?; tail -c 400 gpurun_out/r06k_bench_c4.json; exit $rc
