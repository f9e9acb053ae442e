#!/bin/bash
# A/B of library variants on bench configs: LIBS="a b" (libpa_<a>.so; "base" = libpa.so), CONFIGS="c2 c3"
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
OUT=$R/gpurun_out/ab_$1
mkdir -p $OUT
cd $R
for rep in 1 2; do
for c in $CONFIGS; do
  for l in $LIBS; do
    lib=$P/libpa_$l.so; [ "$l" = base ] && lib=$P/libpa.so
    PA_LIBRARY=$lib timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-traffic $BENCH_ARGS > $OUT/$c.$l.json 2> $OUT/$c.$l.err || { tail -3 $OUT/$c.$l.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$c.$l.json')); print('$c $l', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],3), 'ms')"
  done
done
done
