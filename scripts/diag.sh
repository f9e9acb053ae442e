#!/bin/bash
# Diagnosis of one bench config on the GPU box: the PA_STATS counters of one
# pass (libpa_stats.so) and the timing dissection by phase (libpa_dissect.so,
# PA_DBG_MODE: 13 packing, 14 one seed round, 10 seeds, 11 walk, 12 no second
# walk; results invalid by design), then any env variants of libpa.so.
#   CFG=c2mix MODES="13 14 10 11 12 0" VARIANTS="PA_LANE_MAXPEND=48" bash scripts/diag.sh <tag>
# (BARGS: more bench arguments, e.g. "--read-len 176")
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
OUT=$R/gpurun_out/diag_$1
mkdir -p $OUT
cd $R
B="python bench.py --config $CFG --no-cpu-baseline --no-traffic --no-e2e $BARGS"
PA_LIBRARY=$P/libpa_stats.so timeout -k 10 300 $B --steps 1 --warmup 0 > $OUT/stats.json 2> $OUT/stats.err || { tail -3 $OUT/stats.err; exit 1; }
grep pa_stats $OUT/stats.err | tail -5
for m in $MODES; do
  PA_LIBRARY=$P/libpa_dissect.so PA_DBG_MODE=$m timeout -k 10 300 $B --steps 20 --warmup 3 > $OUT/m$m.json 2> $OUT/m$m.err || { tail -3 $OUT/m$m.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/m$m.json')); r=d['roofline']
print('mode $m pass', round(r['algorithmic']['survey_8d']['pass_ms'],3), {k: round(v,3) for k, v in r['per_rank'][0]['kernels_ms'].items() if v > 0.02})"
done
for v in $VARIANTS; do
  env ${v//,/ } timeout -k 10 300 $B --steps 20 --warmup 3 > $OUT/v.json 2> $OUT/v.err || { tail -3 $OUT/v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/v.json')); r=d['roofline']
print('$v', round(d['value']/1e6,1), 'Mreads/s pass', round(r['algorithmic']['survey_8d']['pass_ms'],3), {k: round(v,3) for k, v in r['per_rank'][0]['kernels_ms'].items() if v > 0.02})"
done
