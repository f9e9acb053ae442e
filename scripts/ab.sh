#!/bin/bash
# A/B of library builds on bench configs (the one A/B launcher):
#   LIBS="base x" CONFIGS="c2 c2mix" REPS=2 BENCH_ARGS="..." bash scripts/ab.sh <tag>
# libpa_<x>.so next to libpa.so ("base" = libpa.so itself); prints reads/s and the
# align-pass / per-kernel times of every (config, library) pair.
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
OUT=$R/gpurun_out/ab_$1
mkdir -p $OUT
cd $R
for rep in $(seq 1 ${REPS:-2}); do
for c in $CONFIGS; do
  for l in $LIBS; do
    lib=$P/libpa_$l.so; [ "$l" = base ] && lib=$P/libpa.so
    PA_LIBRARY=$lib timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-e2e $BENCH_ARGS > $OUT/$c.$l.json 2> $OUT/$c.$l.err || { tail -3 $OUT/$c.$l.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/$c.$l.json')); r=d['roofline']
print('$c $l', round(d['value']/1e6,1), 'Mreads/s, pass', round(r['algorithmic']['survey_8d']['pass_ms'],3), 'ms,', {k: round(v['ms_avg'],3) for k, v in r['kernels'].items()})"
  done
done
done
