#!/bin/bash
# C5 index build under different build settings (PA_CLI_TIMING phases):
#   VARIANTS="PA_BUILD_RUN=16 PA_BUILD_RUN=4" bash scripts/c5_build_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c5ab_$1
mkdir -p $OUT
cd $R
for v in $VARIANTS; do
  tag=$(echo "$v" | tr ':=,' '___')
  env PA_CLI_TIMING=1 ${v//,/ } timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-traffic --no-e2e > $OUT/$tag.json 2> $OUT/$tag.err || { tail -3 $OUT/$tag.err; exit 1; }
  echo "$v: $(grep -o 'index [0-9.]*s (first build [0-9.]*s, align-side view [0-9.]*s)' $OUT/$tag.err)"
done
