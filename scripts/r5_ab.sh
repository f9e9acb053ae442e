#!/bin/bash
# round-5 step: parity subset on the current libpa.so, then an A/B of library variants
#   TESTS="..." LIBS="r4 x base" CONFIGS="c2 c5" bash scripts/r5_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$1; mkdir -p $OUT; cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-500} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
REPS=${REPS:-1} bash scripts/ab.sh $1
