#!/bin/bash
# Index build of one bench config under rocprofv3 --kernel-trace --stats
# (per-kernel build times) plus the [pa_build] phase line:
#   scripts/build_trace.sh c4 [extra bench args]
set -o pipefail
CFG=${1:-c4}
shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${CFG}_build_trace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PA_CLI_TIMING=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $R/bench.py --config $CFG --reads-per-gpu 1000000 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic --no-e2e "$@" > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
python3 $R/profiles/rocpd_summary.py $(find $OUT/trace -name "*.db" | head -1) > $OUT/kernel_stats.txt && rm -rf $OUT/trace
