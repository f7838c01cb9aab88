#!/bin/bash
# r05aa: L2 hit rate per GEMM / attention instance in the UNet forward (rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum, one
# pass, kernel-trace only) -- whether the in-context operand intake is served by the XCD's L2 or from the Infinity
# Cache / HBM
cd "$(dirname "$0")/.."
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/fdprof/tcc
rm -rf $D; mkdir -p $D
(cd /tmp && timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $D -o run \
   -- python3 $R/scripts/pmc_work.py --what unet > $R/gpurun_out/r05aa_tcc.log 2>&1)
rc=$?; echo "pmc rc=$rc"; tail -2 $R/gpurun_out/r05aa_tcc.log; [ $rc -eq 0 ] || exit $rc
for f in "gemm_kernel" "gemm8_kernel" "256ELi160" "256ELi128" "128ELi160" "flash_attn_d64" "conv_halo" "gn_apply"; do
  python3 probes/pmc_agg.py $D "$f"
done | tee gpurun_out/r05aa_tcc_by_kernel.jsonl
