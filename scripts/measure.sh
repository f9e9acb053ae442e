#!/bin/bash
# Round measurement of one bench config on the GPU box:
#   1. the bench line (CPU baseline + parity sample + the in-run counter pass:
#      fabric traffic and SQ shares per align kernel, saved with --profile-dir)
#   2. rocprofv3 --kernel-trace --stats of the same workload (no CPU baseline),
#      summarised by profiles/rocpd_summary.py
# usage: bash scripts/measure.sh <tag> <config> [bench args...]
# then (in the build container): python scripts/save_measure.py <tag> [name]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; CFG=$2; shift 2
OUT=$R/gpurun_out/ms_$TAG
mkdir -p $OUT
echo "$CFG $*" > $OUT/args
cd $R
timeout -k 10 1100 python bench.py --config $CFG --profile-dir $OUT "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
echo bench done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $R/bench.py --config $CFG --no-cpu-baseline --no-traffic --no-e2e "$@" > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
# summarised here, the database dropped (gpurun_out/ must stay under 64 MiB)
python3 $R/profiles/rocpd_summary.py $(find $OUT/trace -name "*.db" | head -1) > $OUT/kernel_stats.txt && rm -rf $OUT/trace
echo trace done
