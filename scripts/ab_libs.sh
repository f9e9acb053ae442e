#!/bin/bash
# A/B of library variants on bench configs, interleaved (bench lines without
# CPU baseline / counter pass / e2e):
#   LIBS="base r2u" CONFIGS="c4 c2" bash scripts/ab_libs.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
OUT=$R/gpurun_out/ab_$1
mkdir -p $OUT
for c in $CONFIGS; do
  for rep in 1 2; do
    for l in $LIBS; do
      lib=$P/libpa_$l.so; [ "$l" = base ] && lib=$P/libpa.so
      PA_LIBRARY=$lib timeout -k 10 300 python3 $R/bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-e2e > $OUT/${c}_${l}_$rep.json 2> $OUT/${c}_${l}_$rep.err || { tail -5 $OUT/${c}_${l}_$rep.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$OUT/${c}_${l}_$rep.json')); print('$c $l $rep', round(d['value']/1e9, 4), 'G reads/s; job index', round(d['job_index']['reads_per_s']/1e9, 4), 'lane ms', round(d['roofline']['kernels']['k_align_lane']['ms_avg'], 3))"
    done
  done
done
