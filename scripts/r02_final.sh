#!/bin/bash
# End-of-session measurement on the GPU box: the GPU suite, then measure.sh
# (bench line + kernel trace + SQ pass) for each config given.
# usage: bash scripts/r02_final.sh <suffix> [tests] <config>...
set -o pipefail
R=$GRAFT_REPO_ROOT
SUF=$1; shift
cd $R
mkdir -p gpurun_out
if [ "$1" = tests ]; then
  shift
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1 || { tail -5 gpurun_out/gpu_tests_final.log; exit 1; }
  echo tests done
fi
for c in "$@"; do
  bash scripts/measure.sh ${c}_$SUF $c || exit 1
  echo "$c measured"
done
