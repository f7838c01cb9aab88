#!/bin/bash
# GroupNorm apply launch shape in the VAE decode (FD_GN_APPLY_U vectors in flight per thread, FD_GN_APPLY_BLOCKS).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/gn_env.jsonl
for rep in 1 2; do
  AB_TAG=base timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/gn_env.jsonl || exit $?
  AB_TAG=u8 FD_GN_APPLY_U=8 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/gn_env.jsonl || exit $?
  AB_TAG=b2048 FD_GN_APPLY_BLOCKS=2048 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/gn_env.jsonl || exit $?
  AB_TAG=u8b2048 FD_GN_APPLY_U=8 FD_GN_APPLY_BLOCKS=2048 timeout -k 10 300 python scripts/vae_ab.py >> gpurun_out/gn_env.jsonl || exit $?
done
python - <<'PY'
import json
for l in open("gpurun_out/gn_env.jsonl"):
    d = json.loads(l); print(d.get("AB_TAG"), d["decode_ms_median"], d["eager_kind_ms"])
PY
