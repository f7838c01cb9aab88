#!/bin/bash
# End-of-round PMC evidence on the current tree: UNet (bf16) and UNet (use_fp8, e4m3 MFMA) traffic passes ->
# profiles' traffic files for bench.py's roofline.traffic, and the VAE decode counter report.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/r02_prof.sh unet r03_unet_pmc > gpurun_out/r03_unet_prof.log 2>&1; rc=$?; tail -2 gpurun_out/r03_unet_prof.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/traffic_from_pmc.py gpurun_out/r03_unet_pmc.json gpurun_out/r03_gemm_traffic.json gemm > /dev/null || exit 1
bash scripts/r02_prof.sh unet_fp8 r03_unet_fp8_pmc > gpurun_out/r03_unet_fp8_prof.log 2>&1; rc=$?; tail -2 gpurun_out/r03_unet_fp8_prof.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/traffic_from_pmc.py gpurun_out/r03_unet_fp8_pmc.json gpurun_out/r03_gemm_traffic_fp8.json gemm_e4m3 > /dev/null || exit 1
bash scripts/r02_prof.sh vae r03_vae_pmc > gpurun_out/r03_vae_prof.log 2>&1; rc=$?; tail -2 gpurun_out/r03_vae_prof.log; [ $rc -eq 0 ] || exit $rc
ls gpurun_out/r03_*pmc* gpurun_out/r03_gemm_traffic*
