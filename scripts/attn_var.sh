#!/bin/bash
# flash d64 variants (FD_FLASH_WAVES x FD_FLASH_QPW): correctness vs torch, then graph-timed UNet shapes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/attn_var.jsonl; : > $out
S="2x20x1024x1024 2x10x4096x4096 2x20x1024x77 2x10x4096x77 26x20x1024x1024 26x10x4096x77"
for v in "4 32" "4 16" "8 16" "2 16"; do
  set -- $v
  FD_FLASH_WAVES=$1 FD_FLASH_QPW=$2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash_attn and not d512" > gpurun_out/attn_var_test.log 2>&1
  rc=$?; echo "waves $1 qpw $2: $(tail -1 gpurun_out/attn_var_test.log)"; [ $rc -eq 0 ] || exit $rc
  FD_FLASH_WAVES=$1 FD_FLASH_QPW=$2 timeout -k 10 120 python scripts/attn_probe.py $S >> $out 2>/dev/null || exit $?
done
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/attn_var.jsonl')]
for sh in dict.fromkeys(r['shape'] for r in rows):
    print(f"{sh:22s}", ' | '.join(f"w{r['FD_FLASH_WAVES']}q{r['FD_FLASH_QPW']}: {r['us']}" for r in rows if r['shape']==sh))
PY
