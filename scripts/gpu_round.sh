#!/bin/bash
# GPU tests + bench lines for a tag; usage: bash scripts/gpu_round.sh <tag> [configs...]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/r_$TAG
mkdir -p $OUT
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
  tail -2 $OUT/gputest.log
fi
for c in "$@"; do
  timeout -k 10 900 python bench.py --config $c $BENCH_ARGS > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); r=d['roofline']; print('$c', round(d['value']/1e6,1), 'Mreads/s', round(r['kernel_ms'],3), 'ms', 'frac', round(r['frac'],3), 'measured', r['measured_frac'] and round(r['measured_frac'],3), 'lines', r['lines_per_read'] and round(r['lines_per_read'],2), 'exact', (d.get('parity_sample') or {}).get('bit_exact'))"
done
