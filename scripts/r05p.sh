#!/bin/bash
# r05p: nt weight-operand loads A/B (wld2 build), then the kernel trace of the C2 bench on the write-through tree
# (step window, GEMM instances in context, roofline check) and the UNet PMC passes -> the roofline.traffic file
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=$PWD/faithdiff-dev_amd/fdhip
bash scripts/run.sh r05p "abv=2;FD_LIB_PATH=$P/libfaithdiff_hip.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wld2.so" || exit $?
bash scripts/run.sh r05p trace pmc=unet || exit $?
python3 scripts/traffic_from_pmc.py gpurun_out/r05p_unet_pmc.json gpurun_out/r05p_gemm_traffic.json || exit $?
