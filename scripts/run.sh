#!/bin/bash
# Parameterised GPU-box runner (replaces the round-specific r0x_* scripts).  Each phase runs under its own time
# limit; the first failing phase ends the run (no GPU step after a failure).  Outputs: gpurun_out/<tag>_<phase>.*
#
#   scripts/run.sh <tag> <phase> [<phase> ...]
#     smoke                     __graft_entry__.smoke()
#     tests[=<pytest -k expr>]  the -m gpu suite (-v), parity metrics to gpurun_out/<tag>_parity_metrics.json
#     tfile=<path>[:<-k expr>]  one GPU test file
#     bench[=<args>]            bench.py line (args with ',' for spaces, e.g. bench=--fp8,--no-c3)
#     trace                     rocprofv3 kernel trace of the C2 bench: step window, GEMM instances, roofline check
#     pmc=<unet|unet_fp8|vae|attn>   counter passes (scripts/prof.sh)
#     probe=<script>[,args]     a python probe / measurement script
#     ab=<reps>;<envA>;<envB>   alternating bench A/B (knob env per arm, e.g. ab=2;X=0;FD_GEMM8_W128=0)
# Knob overrides (FD_*) reach bench.py / probes through fdhip.knobs.apply_env(); the product never reads them.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=$1; shift
for ph in "$@"; do
  name=${ph%%=*}; arg=${ph#*=}; [ "$arg" = "$ph" ] && arg=""
  out=gpurun_out/${TAG}_${name}
  echo "== $ph"
  case $name in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out.log 2>&1; rc=$?; tail -2 $out.log ;;
    tests)
      export FD_PARITY_METRICS=$PWD/gpurun_out/${TAG}_parity_metrics.json; rm -f $FD_PARITY_METRICS
      if [ -n "$arg" ]; then K=(-k "$arg"); else K=(); fi
      timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ "${K[@]}" > $out.log 2>&1
      rc=$?; tail -4 $out.log ;;
    tfile)
      f=${arg%%:*}; k=${arg#*:}; [ "$k" = "$arg" ] && k=""; out=gpurun_out/${TAG}_$(basename $f .py)
      export FD_PARITY_METRICS=$PWD/${out}_parity_metrics.json; rm -f $FD_PARITY_METRICS
      if [ -n "$k" ]; then K=(-k "$k"); else K=(); fi
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$f" "${K[@]}" > $out.log 2>&1
      rc=$?; tail -8 $out.log ;;
    bench)
      [ -n "$arg" ] && out=${out}_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_' | sed 's/_*$//')
      timeout -k 10 600 python bench.py ${arg//,/ } > $out.json 2> $out.err; rc=$?; tail -c 700 $out.json ;;
    trace)
      bash scripts/trace.sh $TAG > $out.log 2>&1; rc=$?; tail -30 $out.log ;;
    pmc)
      bash scripts/prof.sh $arg ${TAG}_${arg}_pmc > $out.log 2>&1; rc=$?; tail -3 $out.log ;;
    probe)
      sc=${arg%%,*}; out=gpurun_out/${TAG}_$(basename $sc .py)
      timeout -k 10 400 python -u ${arg//,/ } > $out.log 2>&1; rc=$?; tail -25 $out.log ;;
    ab|abv|abf)  # abv: with the VAE decode leg (prints vae_decode_ms too); abf: the use_fp8 model (--fp8)
      IFS=';' read -r reps rest <<< "$arg"; IFS=';' read -ra arms <<< "$rest"; : > $out.txt
      if [ $name = abv ]; then VA=""; else VA="--no-vae"; fi
      if [ $name = abf ]; then VA="$VA --fp8"; fi
      for r in $(seq $reps); do for e in "${arms[@]}"; do
        env $e timeout -k 10 300 python bench.py --no-cpu-baseline $VA --no-c3 --no-pipeline --steps 30 > $out.run 2>&1 || { rc=$?; break 2; }
        echo "$e $(tail -1 $out.run | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("roofline", {}).get("frac"), d.get("vae_decode_ms"))')" | tee -a $out.txt
        rc=0
      done; done ;;
    *) echo "unknown phase $ph"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || { echo "phase $ph failed rc=$rc"; exit $rc; }
done
