#!/bin/bash
# VAE decode: the N = 128 convs at 1024^2 on gemm8 256x128 (one 8-wave WG per CU) vs the 4-wave family's 128-row
# tiles (two WGs per CU, so one tile's prologue / epilogue overlaps the other's main loop).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/vae_tile.jsonl
for rep in 1 2; do
  AB_TAG=base timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_tile.jsonl || exit $?
  AB_TAG=g8off FD_GEMM8=0 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_tile.jsonl || exit $?
  AB_TAG=g8off_c128 FD_GEMM8=0 FD_GEMM_CFG=0 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_tile.jsonl || exit $?
  AB_TAG=g8off_c128ns3 FD_GEMM8=0 FD_GEMM_CFG=0 FD_GEMM_NS=3 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/vae_tile.jsonl || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/vae_tile.jsonl"):
    d = json.loads(l)
    n128 = [t for t in d["top"] if "N=128 " in t[0]]
    print(d.get("AB_TAG"), d["decode_ms_median"], d["eager_kind_ms"], n128)
PY
