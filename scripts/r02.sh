#!/bin/bash
# Round-2 GPU session driver.  Usage: scripts/r02.sh STEP [STEP ...]
# Every GPU step runs under its own time limit; a fault / abort / timeout (rc other than 0 / 1) ends the script
# so no further GPU work starts in that call.  Logs: gpurun_out/<step>.log
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
run() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
for step in "$@"; do
  case $step in
    t_new) run t_new 900 $PYT tests/test_tile_parallel_gpu.py tests/test_pipeline_gpu.py -s ;;
    t_c2) run t_c2 600 $PYT tests/test_pipeline_gpu.py -s -k c2_headline ;;
    t_fp8) run t_fp8 900 $PYT tests/test_fp8_gpu.py -s ;;
    t_unet) run t_unet 900 $PYT tests/test_unet_gpu.py -s ;;
    t_kern) run t_kern 900 $PYT tests/test_kernels_gpu.py tests/test_gemm8_gpu.py tests/test_ln_fold_gpu.py tests/test_clip_gpu.py ;;
    allgpu) run allgpu 1100 $PYT tests -q ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    bench_quick) run bench_quick 600 python bench.py --no-cpu-baseline --no-c3 ;;
    bench_c3) run bench_c3 600 python bench.py --workload c3 --no-cpu-baseline ;;
    bench_fp8) run bench_fp8 600 python bench.py --fp8 --no-cpu-baseline --no-c3 --no-pipeline ;;
    rehearsal) FD_BENCH_REHEARSAL=1 run rehearsal 600 python bench.py --gpus 2 --no-cpu-baseline --no-pipeline --no-roofline --no-vae --c3-steps 2 --steps 5 ;;
    prof) run prof 600 bash scripts/r02_trace.sh ;;
    pmc_unet) run pmc_unet 700 bash scripts/r02_prof.sh unet r02_unet_pmc ;;
    pmc_vae) run pmc_vae 700 bash scripts/r02_prof.sh vae r02_vae_pmc ;;
    pmc_fp8) run pmc_fp8 700 bash scripts/r02_prof.sh unet_fp8 r02_unet_fp8_pmc ;;
    vendor) run vendor 300 python scripts/vendor_compare.py ;;
    pmc_attn) run pmc_attn 700 bash scripts/r02_prof.sh attn r02_attn_pmc ;;
    *) echo "unknown step $step"; exit 3 ;;
  esac
done
