#!/bin/bash
# A/B of an alternative library build (FD_LIB_PATH) against the product library on the same box, interleaved
cd "$(dirname "$0")/.."
ALT=${ALT:-$(pwd)/faithdiff-dev_amd/fdhip/diag/lib_sp.so}
SH="2048x10240x1280:geglu 2048x3840x1280 conv64x64x640x640 conv128x128x320x320 8192x8192x8192 conv256x512x256x256 conv128x256x512x512 conv512x1024x128x128"
out=gpurun_out/sp_ab.jsonl; : > $out
for r in 1 2; do
  PROBE_TAG=base timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
  PROBE_TAG=alt FD_LIB_PATH=$ALT timeout -k 10 200 python scripts/gemm_probe.py $SH >> $out 2>/dev/null || exit $?
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 --no-pipeline --no-roofline > gpurun_out/sp_b_base$r.log 2>&1 || exit $?
  FD_LIB_PATH=$ALT timeout -k 10 300 python bench.py --no-cpu-baseline --no-c3 --no-pipeline --no-roofline > gpurun_out/sp_b_alt$r.log 2>&1 || exit $?
done
python - <<'PY'
import json,collections
d=collections.defaultdict(list)
for l in open("gpurun_out/sp_ab.jsonl"):
    if l.startswith("{"):
        j=json.loads(l); d[(j["shape"], j.get("PROBE_TAG",""))].append(j["us"])
for (sh,tag),v in sorted(d.items()): print(f"{sh:28s} {tag:5s} {min(v):9.2f} us")
for n in ("base1","alt1","base2","alt2"):
    j=json.loads([l for l in open(f"gpurun_out/sp_b_{n}.log") if l.startswith('{"metric"')][-1])
    print(n, j["ms_per_step"], j.get("vae_decode_ms"))
PY
