#!/bin/bash
# r05g: d512 split parity (generalised kernel), UNet PMC passes -> the roofline.traffic file, and the 2-rank
# rehearsal bench line (both ranks on cuda:0 over gloo) carrying the SCALE diagnostics
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05g "tfile=tests/test_kernels_gpu.py:d512" "tfile=tests/test_pipeline_gpu.py:vae" pmc=unet || exit $?
python3 scripts/traffic_from_pmc.py gpurun_out/r05g_unet_pmc.json gpurun_out/r05g_gemm_traffic.json || exit $?
FD_BENCH_REHEARSAL=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline \
  > gpurun_out/r05g_bench_rehearsal_2rank.json 2> gpurun_out/r05g_bench_rehearsal_2rank.err || exit $?
tail -c 1500 gpurun_out/r05g_bench_rehearsal_2rank.json
# halo-conv K-loop diagnostics (wrong-answer timing builds: 1 no DMA waits, 2 no MFMAs, 5 LDS + MFMA only, 8 no
# barriers) against the product build
for lib in fdhip/libfaithdiff_hip.so fdhip/ab/libfaithdiff_hip_hd1.so fdhip/ab/libfaithdiff_hip_hd2.so fdhip/ab/libfaithdiff_hip_hd5.so fdhip/ab/libfaithdiff_hip_hd8.so; do
  FD_LIB_PATH=$PWD/faithdiff-dev_amd/$lib timeout -k 10 300 python probes/conv_ab.py > gpurun_out/r05g_diag_$(basename $lib .so).jsonl 2>&1 || exit $?
done
