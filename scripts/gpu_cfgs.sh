#!/bin/bash
# Bench lines of several configs with one library (counter pass off):
#   CONFIGS="c2k63 c2l250" LIB=base BENCH_ARGS="..." bash scripts/gpu_cfgs.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
P=$R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
OUT=$R/gpurun_out/cfg_$1
mkdir -p $OUT
cd $R
l=${LIB:-base}
lib=$P/libpa_$l.so; [ "$l" = base ] && lib=$P/libpa.so
for c in $CONFIGS; do
  PA_LIBRARY=$lib timeout -k 10 ${CFG_LIMIT:-300} python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e $BENCH_ARGS > $OUT/$c.json 2> $OUT/$c.err || { tail -5 $OUT/$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$c.json')); r=d['roofline']
print('$c', round(d['value']/1e6,1), 'Mreads/s frac', r.get('frac'), 'kernel', round(r['algorithmic']['kernel_ms'],3), 'ms,', {k: round(v['ms_avg'],3) for k, v in r['kernels'].items()})"
done
