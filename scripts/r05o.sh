#!/bin/bash
# r05o: sc1 write-through output stores (with the wait states behind the 16-B inline-asm store) and the fp16
# pre-scaled self-attention (fd_flash_attn_pre, FD_FLASH_PRE): smoke, the C2 step / VAE decode A/B against plain
# stores (wt0) and sc1 nt (wt4), the FD_FLASH_PRE A/B, the full GPU suite, the bench line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
P=$PWD/faithdiff-dev_amd/fdhip
bash scripts/run.sh r05o smoke || exit $?
bash scripts/run.sh r05o "abv=2;FD_LIB_PATH=$P/libfaithdiff_hip.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wt0.so;FD_LIB_PATH=$P/ab/libfaithdiff_hip_wt4.so" || exit $?
mv gpurun_out/r05o_abv.txt gpurun_out/r05o_store_ab.txt
bash scripts/run.sh r05o "ab=2;FD_FLASH_PRE=0;FD_FLASH_PRE=1" || exit $?
mv gpurun_out/r05o_ab.txt gpurun_out/r05o_flash_pre_ab.txt
bash scripts/run.sh r05o tests || exit $?
bash scripts/run.sh r05o bench || exit $?
