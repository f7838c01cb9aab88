#!/bin/bash
# r06g: the C2 headline / teacher-forced parity tests with the UNet in bf16 (product default) and in fp16 (the
# reference's own UNet dtype)
cd "$(dirname "$0")/.."
bash scripts/run.sh r06g "tfile=tests/test_pipeline_gpu.py:c2_"
