#!/bin/bash
# A/B of environment settings (and libraries) on bench configs:
#   VARIANTS="base:PA_BLOOM_MB=64 base:PA_BLOOM_MB=128 old:" CONFIGS="c2 c2rc" bash scripts/ab_env.sh <tag>
# each variant is <lib>:<VAR=value,...> (lib "base" = libpa.so, else libpa_<lib>.so)
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
OUT=$R/gpurun_out/abe_$1
mkdir -p $OUT
cd $R
for rep in $(seq 1 ${REPS:-1}); do
for c in $CONFIGS; do
  for v in $VARIANTS; do
    l=${v%%:*}; e=${v#*:}
    lib=$P/libpa_$l.so; [ "$l" = base ] && lib=$P/libpa.so
    tag=$(echo "$c.$v" | tr ':=,' '___')
    env PA_LIBRARY=$lib ${e//,/ } timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-e2e $BENCH_ARGS > $OUT/$tag.json 2> $OUT/$tag.err || { tail -3 $OUT/$tag.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/$tag.json')); r=d['roofline']
print('$c $v', round(d['value']/1e6,1), 'Mreads/s, pass', round(r['algorithmic']['pass_ms'],3), 'ms,', {k: round(v['ms_avg'],3) for k, v in r['kernels'].items()})"
  done
done
done
