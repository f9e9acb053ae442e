#!/bin/bash
# FETCH_SIZE calibration + random-line rates (profiles/fetch_calib.hip); usage: bash scripts/calib.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/calib_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -k 10 120 $R/profiles/fetch_calib > $OUT/calib.json 2> $OUT/calib.err || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc -o run -- $R/profiles/fetch_calib > /dev/null 2> $OUT/pmc.err || exit 1
python3 $R/profiles/rocpd_summary.py $OUT/pmc/run_results.db > $OUT/calib_pmc.txt || exit 1
echo done
