# L2 requests per phase of the lane kernel: the PA_DISSECT build, dbg modes
# (13: stop after the packing, 14: one seed round, 10: stop after the seeds, 11: after the walk, 12: no second walk, 0: all), one PMC pass each
export PA_LIBRARY=$GRAFT_REPO_ROOT/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/libpa_dissect.so
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-10 11 12 0}; do
  PA_DBG_MODE=$m timeout -k 10 240 rocprofv3 --kernel-trace --pmc TCC_REQ_sum TCC_BUSY_avr TA_BUSY_avr GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/pmcph/m$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $GRAFT_REPO_ROOT/gpurun_out/pmcph_m$m.log 2>&1 || exit 1
done
echo done
