#!/bin/bash
# End-of-round evidence on the current tree: the bench under rocprofv3 --kernel-trace --stats (step window, GEMM
# instances, roofline cross-check), then the UNet PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) and bench.py's
# traffic file from them.  Each step bounded by its own timeouts (inside the called scripts).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/r02_trace.sh > gpurun_out/r02f_trace.log 2>&1; rc=$?; tail -3 gpurun_out/r02f_trace.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r02_prof.sh unet r02f_unet_pmc > gpurun_out/r02f_unet_prof.log 2>&1; rc=$?; tail -3 gpurun_out/r02f_unet_prof.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/traffic_from_pmc.py gpurun_out/r02f_unet_pmc.json gpurun_out/r02f_gemm_traffic.json
