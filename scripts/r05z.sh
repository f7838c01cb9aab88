#!/bin/bash
# r05z: planner knob re-check, part 2 (GroupNorm apply grid, flash attention form / order, tile walks) on the C2 step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r05z "ab=2;FD_NONE=0;FD_GN_APPLY_U=8;FD_GN_APPLY_BLOCKS=2048;FD_GN_APPLY_BLOCKS=512;FD_FLASH_QPW=32;FD_FLASH_SWZ=0;FD_GEMM_SWZ=0;FD_GEMM256_MIN_TILES=128;FD_GN_MIN_CHUNKS=128" || exit $?
