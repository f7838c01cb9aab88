#!/bin/bash
# flash d64 K/V ring depth A/B: libraries built with -DFLASH_NBUF=4 / 6 (exp_nb*.so) against the in-tree 3
cd "$(dirname "$0")/.."
S="2x20x1024x1024 2x10x4096x4096 2x20x1024x77 2x10x4096x77 26x20x1024x1024 26x10x4096x77"
for lib in "" exp/nb4.so exp/nb6.so; do
  for q in 16 32; do
    echo "lib=${lib:-nb3} qpw=$q"
    FD_LIB_PATH=${lib:+$PWD/$lib} FD_FLASH_QPW=$q timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_flash_attn and not d512" > gpurun_out/nb_test.log 2>&1 || { tail -5 gpurun_out/nb_test.log; exit 1; }
    FD_LIB_PATH=${lib:+$PWD/$lib} FD_FLASH_QPW=$q timeout -k 10 100 python scripts/attn_probe.py $S 2>/dev/null | python -c "import sys,json; print(' | '.join(f\"{d['shape']}: {d['us']}\" for d in map(json.loads, sys.stdin)))" || exit 1
  done
done
