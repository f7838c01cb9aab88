#!/bin/bash
# One GPU session: parity tests, smoke, bench. Each GPU step has its own time limit; a fault / abort /
# timeout ends the script (no further GPU work); an ordinary test failure (rc 1) does not.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name" ; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    kernels) run kernels 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -p no:cacheprovider ;;
    unet) run unet 900 python -m pytest tests/test_unet_gpu.py -m gpu -q -s -p no:cacheprovider ;;
    pipeline) run pipeline 1000 python -m pytest tests/test_pipeline_gpu.py -m gpu -q -s -p no:cacheprovider ;;
    allgpu) run allgpu 1100 python -m pytest tests -m gpu -q -s -p no:cacheprovider ;;
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_nograph) run bench_nograph 600 python bench.py --no-graph --no-cpu-baseline --no-vae --steps 5 ;;
    *) echo "unknown step $step" ;;
  esac
done
