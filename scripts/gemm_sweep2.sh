#!/bin/bash
# Graph-timed GEMM sweep: tile cfg x ring depth x K split (mode 0), then load-only / compute-only modes.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/gemm_sweep2.jsonl; : > $out
SH="2048x1280x1280 2048x1280x5120 2048x3840x1280 2048x10240x1280:geglu conv32x32x1280x1280 8192x640x640 8192x5120x640:geglu conv64x64x640x640 conv128x128x320x320"
for cfg in 0 1 2 3; do for ns in 2 4; do for ks in 1 2; do
  FD_GEMM_CFG=$cfg FD_GEMM_NS=$ns FD_GEMM_KS=$ks timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>gpurun_out/gemm_sweep2.err || exit $?
done; done; done
for cfg in 0 1; do for mode in 1 2; do
  FD_GEMM_CFG=$cfg FD_GEMM_NS=4 FD_GEMM_KS=2 FD_GEMM_MODE=$mode timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>>gpurun_out/gemm_sweep2.err || exit $?
done; done
timeout -k 5 120 python scripts/gemm_probe.py $SH >> $out 2>>gpurun_out/gemm_sweep2.err || exit $?
python - <<'PY'
import json
rows=[json.loads(l) for l in open('gpurun_out/gemm_sweep2.jsonl')]
for shape in dict.fromkeys(r['shape'] for r in rows):
    rs=[r for r in rows if r['shape']==shape]
    dflt=[r for r in rs if 'FD_GEMM_CFG' not in r]
    m0=sorted((r for r in rs if r.get('FD_GEMM_MODE','0')=='0' and 'FD_GEMM_CFG' in r), key=lambda r:r['us'])
    print(shape, 'default', dflt[0]['us'] if dflt else None, '| best', ' '.join(f"c{r['FD_GEMM_CFG']}n{r['FD_GEMM_NS']}k{r['FD_GEMM_KS']}:{r['us']}" for r in m0[:5]))
    print('   modes', ' '.join(f"c{r['FD_GEMM_CFG']}m{r['FD_GEMM_MODE']}:{r['us']}" for r in rs if r.get('FD_GEMM_MODE','0')!='0'))
PY
