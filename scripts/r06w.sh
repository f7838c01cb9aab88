#!/bin/bash
# r06w: GroupNorm statistics chunk floor (FD_GN_MIN_CHUNKS, 256 default) -- more chunks = more workgroups for the
# statistics pass and the concat + statistics launch, a longer fold
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06w "abv=3;FD_AB_ARM=256;FD_GN_MIN_CHUNKS=512;FD_GN_MIN_CHUNKS=1024"
