# instruction counts per phase: stats build, dbg modes, one PMC pass each
export PA_LIBRARY=$GRAFT_REPO_ROOT/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/libpa_stats.so
cd /tmp && export TMPDIR=/tmp
for m in 2 3 4 0; do
  PA_DBG_MODE=$m timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d $GRAFT_REPO_ROOT/gpurun_out/pmcph/m$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmcph_m$m.log 2>&1 || exit 1
done
echo done
