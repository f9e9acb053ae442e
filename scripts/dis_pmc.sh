set -o pipefail
P=$GRAFT_REPO_ROOT/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
for m in 13 10 11 12 0; do
  PA_LIBRARY=$P/libpa_dis.so PA_DBG_MODE=$m timeout -k 10 200 python scripts/pmc_diag.py c2mix SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAVES SQ_INSTS_SMEM > gpurun_out/dis_pmc_$m.json 2> gpurun_out/dis_pmc_$m.err || exit 1
  echo mode $m done
done
