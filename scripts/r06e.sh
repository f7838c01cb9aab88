#!/bin/bash
# r06e: the sigmoid-logit GELU: GEGLU / GELU / UNet parity tests and smoke on it; C2 step A/B
# against the A-S erf form (build-time FD_GELU_AS=1, fdhip/ab/); then the in-context probe (r06d.sh)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
AB=$PWD/faithdiff-dev_amd/fdhip/ab
bash scripts/run.sh r06e "tests=geglu or gelu or unet" smoke "ab=3;FD_LIB_PATH=$AB/libfaithdiff_hip_gelu_as.so;FD_AB_ARM=sigmoid" || exit $?
bash scripts/r06d.sh
