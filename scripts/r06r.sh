#!/bin/bash
# r06r: C2 teacher-forced eps against the fp32 oracle for the bf16, fp16 and use_fp8 (e4m3 MFMA) UNets
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash scripts/run.sh r06r "tfile=tests/test_pipeline_gpu.py:teacher_forced"
