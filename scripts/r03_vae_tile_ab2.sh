#!/bin/bash
# VAE decode: the 256/512-channel convs on gemm256 (one 256x256 WG per CU, default) vs the 4-wave 128x128 tiles
# (two WGs per CU; FD_GEMM256=0 FD_GEMM8=0) vs gemm8 256x128 (FD_GEMM256=0).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/vae_tile2.jsonl
for rep in 1 2; do
  AB_TAG=base timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_tile2.jsonl || exit $?
  AB_TAG=all4w FD_GEMM256=0 FD_GEMM8=0 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_tile2.jsonl || exit $?
  AB_TAG=g256off FD_GEMM256=0 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_tile2.jsonl || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/vae_tile2.jsonl"):
    d = json.loads(l)
    print(d.get("AB_TAG"), d["decode_ms_median"], d["eager_kind_ms"])
    for t in d["top"]:
        print("    ", t)
PY
