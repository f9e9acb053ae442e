#!/bin/bash
# A/B: C4 with the table at 4 (default) vs 2 slots per genome window (PA_CAP_MULT=2):
# build time, job-index and serving-index align rates
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_cap
mkdir -p $OUT
for m in 4 2; do
  PA_CAP_MULT=$m timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-traffic --no-e2e > $OUT/c4_cap$m.json 2> $OUT/c4_cap$m.err || exit 1
done
