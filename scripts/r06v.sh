#!/bin/bash
# r06v: with the concat now writing norm1's statistics, re-check how wide an input the halo conv's GroupNorm fold
# should take (FD_HALO_GN_CIN_MAX: 640 default, 960 / 1280 cover the 64^2-level concats)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06v "ab=3;FD_AB_ARM=640;FD_HALO_GN_CIN_MAX=960;FD_HALO_GN_CIN_MAX=1280"
