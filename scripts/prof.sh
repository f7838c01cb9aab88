#!/bin/bash
# rocprofv3 evidence for one scripts/pmc_work.py workload: a kernel-trace pass (durations), then separate PMC
# passes (FETCH_SIZE; WRITE_SIZE; SQ group) -- kernel-trace only, never a runtime / sys trace domain, one
# counter group per pass within the gfx950 slot limits (8 SQ, 4 TCC, 2 GRBM).  Then scripts/pmc_report.py.
# Usage: scripts/prof.sh <unet|vae|attn> <tag>     (writes gpurun_out/pmc_<what>/ and gpurun_out/<tag>.json)
cd "$(dirname "$0")/.."
R=$(pwd)
W=$1; TAG=$2
export TMPDIR=/tmp
# raw traces / counter CSVs stay on the box (/tmp: gpurun copies back at most 64 MiB); summaries go to gpurun_out
D=/tmp/fdprof/pmc_$W
rm -rf $D; mkdir -p $D $R/gpurun_out
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run \
   -- python3 $R/scripts/pmc_work.py --what $W > $D/trace.log 2>&1)
rc=$?; echo "trace rc=$rc"; tail -1 $D/trace.log; [ $rc -eq 0 ] || exit $rc
passes="FETCH_SIZE WRITE_SIZE sq1"
[ "$W" = "attn" ] && passes="sq1 sq2 FETCH_SIZE"
for p in $passes; do
  case $p in sq1) C=$SQ1 ;; sq2) C=$SQ2 ;; *) C=$p ;; esac
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $D/$p -o run \
     -- python3 $R/scripts/pmc_work.py --what $W > $D/$p.log 2>&1)
  rc=$?; echo "$p rc=$rc"; tail -1 $D/$p.log; [ $rc -eq 0 ] || exit $rc
done
python3 scripts/pmc_report.py $W $R/gpurun_out/$TAG.json $D
cp $(find $D/trace -name "*kernel_stats.csv" | head -1) $R/gpurun_out/${TAG}_kernel_stats.csv
