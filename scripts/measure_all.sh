#!/bin/bash
# scripts/measure.sh over several configs in one GPU session (the first failure ends it):
#   CONFIGS="c2 c3" ARGS="--no-e2e" bash scripts/measure_all.sh <round tag>
# then in the build container: ROUND=<round> python scripts/save_measure.py <round tag>_<config> <config>
set -o pipefail
for c in $CONFIGS; do
  bash scripts/measure.sh ${1}_$c $c $ARGS || exit 1
  python3 -c "
import json; d=json.load(open('$GRAFT_REPO_ROOT/gpurun_out/ms_${1}_$c/bench.json')); r=d['roofline']
print('$c', round(d['value']/1e9,3), 'G reads/s, frac', r['frac'] and round(r['frac'],3), 'lines/read', r.get('pass_lines_per_read') and round(r['pass_lines_per_read'],2), 'parity', (d.get('parity_sample') or {}).get('bit_exact'))"
done
