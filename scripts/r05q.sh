#!/bin/bash
# r05q: the other workloads on the write-through tree (use_fp8 C2 leg, C4 8K-output, C5 8 images), and the HIP
# runtime's device-memory kernel-argument switch A/B on the C2 step (HIP_FORCE_DEV_KERNARG)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python probes/sdma_prefetch.py > gpurun_out/r05q_sdma_prefetch.jsonl 2>&1 || exit $?
cat gpurun_out/r05q_sdma_prefetch.jsonl
bash scripts/run.sh r05q "ab=2;HIP_FORCE_DEV_KERNARG=0;HIP_FORCE_DEV_KERNARG=1" || exit $?
mv gpurun_out/r05q_ab.txt gpurun_out/r05q_kernarg_ab.txt
timeout -k 10 400 python bench.py --fp8 --no-c3 --no-pipeline --no-cpu-baseline > gpurun_out/r05q_bench_fp8.json 2> gpurun_out/r05q_bench_fp8.err || exit $?
tail -c 600 gpurun_out/r05q_bench_fp8.json
timeout -k 10 500 python bench.py --workload c4 --no-cpu-baseline > gpurun_out/r05q_bench_c4.json 2> gpurun_out/r05q_bench_c4.err || exit $?
tail -c 600 gpurun_out/r05q_bench_c4.json
timeout -k 10 500 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/r05q_bench_c5.json 2> gpurun_out/r05q_bench_c5.err || exit $?
tail -c 600 gpurun_out/r05q_bench_c5.json
