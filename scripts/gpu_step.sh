#!/bin/bash
# One GPU session step list: parity tests, A/B of library builds, the default bench line.
#   TESTS="tests/test_gpu_parity.py ..." LIBS="base r3" CONFIGS="c2 c2mix" DEFAULT=1 bash scripts/gpu_step.sh <tag>
# Every step under its own time limit; the first failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-500} python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
if [ -n "$LIBS" ]; then
  REPS=${REPS:-1} bash scripts/ab.sh $1 || exit 1
fi
if [ -n "$DEFAULT" ]; then
  timeout -k 10 580 python bench.py --gpus 1 --steps 20 --warmup 5 $DEFAULT_ARGS > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_default.json')); r=d['roofline']
print('default', d['config']['workload'][:40], round(d['value']/1e9,3), 'G reads/s frac', r['frac'], 'parity', d.get('parity_sample',{}).get('bit_exact'), 'e2e', (d.get('end_to_end') or {}).get('cli_wall_s'))"
fi
