#!/bin/bash
# (1) the M = 2048 K = 1280 residual-stream projection with / without residual and LN partials (probe, cold weights);
# (2) GroupNorm launch-shape knobs in the bench step (FD_GN_APPLY_BLOCKS, FD_GN_MIN_CHUNKS), interleaved.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/lno_probe.jsonl; : > $out
export PROBE_COPIES=24
[ "${SKIP_PROBE:-0}" = 1 ] || for v in "0 0" "1 0" "1 1"; do set -- $v
  PROBE_RES=$1 PROBE_LNO=$2 timeout -k 5 120 python scripts/gemm_probe.py 2048x1280x1280 2048x1280x5120 >> $out 2>/dev/null || exit $?
done
[ "${SKIP_PROBE:-0}" = 1 ] || cat $out
unset PROBE_COPIES
B="--no-cpu-baseline --no-c3 --no-pipeline --no-roofline --no-vae --steps 40"
for r in 1 2; do
  for cfg in ${GN_CFGS:-"1024,256" "512,256" "1024,64" "256,64"}; do set -- ${cfg/,/ }
    FD_GN_APPLY_BLOCKS=$1 FD_GN_MIN_CHUNKS=$2 timeout -k 10 200 python bench.py $B > gpurun_out/gn_$1_$2_$r.log 2>&1 || exit $?
    python -c "import json; j=json.loads([l for l in open('gpurun_out/gn_$1_$2_$r.log') if l.startswith('{')][-1]); print('apply=$1 chunks=$2 r$r', j['ms_per_step'])"
  done
done
