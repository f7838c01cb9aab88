#!/bin/bash
# A/B on one box, alternated: the M = 2048 projections on gemm8's 64 x 160 one-wave-per-SIMD tile (FD_GEMM_R4=1/2)
# vs the 4-wave gemm.hip kernel (default), C2 step.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do for v in 0 1 2; do
FD_GEMM_R4=$v timeout -k 10 300 python bench.py --no-c3 --no-pipeline --no-cpu-baseline --no-roofline --no-vae --steps 60 > gpurun_out/r4_$v.json 2> gpurun_out/r4_$v.err || exit $?
python -c "import json;d=json.loads(open('gpurun_out/r4_$v.json').read().strip().splitlines()[-1]);print('R4=$v rep$rep', d['ms_per_step'])"
done; done
