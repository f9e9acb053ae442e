#!/bin/bash
# Lane-kernel timing dissection (PA_DISSECT build: stop every read after a phase) and PA_STATS counters.
# usage: bash scripts/dissect.sh <tag> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/dis_$TAG
mkdir -p $OUT
cd $R
P=$R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
for m in 13 14 10 11 12 0; do
  PA_LIBRARY=$P/libpa_dissect.so PA_DBG_MODE=$m timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-traffic "$@" > $OUT/m$m.json 2> $OUT/m$m.err || { tail -3 $OUT/m$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/m$m.json')); print('mode $m', round(d['roofline']['kernel_ms'],3), 'ms')"
done
PA_LIBRARY=$P/libpa_stats.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-traffic "$@" 2>&1 | grep pa_stats | tail -6
