set -e
export TMPDIR=/tmp
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
R=$GRAFT_REPO_ROOT
for p in sq1 sq2; do
  case $p in sq1) C=$SQ1 ;; sq2) C=$SQ2 ;; esac
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d /tmp/pc_$p -o run -- python3 $R/probes/conv_ab.py vae1024_128 > /tmp/pc_$p.log 2>&1)
  python3 $R/probes/pmc_agg.py /tmp/pc_$p conv_halo_kernelIDF16_Li16ELi128ELb0E >> $R/gpurun_out/r04k_halo_pmc.jsonl
done
