#!/bin/bash
# Request-size PMC passes: calibration kernels and the C2 align pass; usage: bash scripts/pmc_c2.sh <tag> [bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/calib -o run -- $R/profiles/fetch_calib > /dev/null 2> $OUT/calib.err || exit 1
python3 $R/profiles/rocpd_summary.py $OUT/calib/run_results.db > $OUT/calib_req.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/req -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic "$@" > $OUT/req.log 2>&1 || exit 1
python3 $R/profiles/rocpd_summary.py $OUT/req/run_results.db > $OUT/req.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_STREAMING_REQ_sum -d $OUT/l2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic "$@" > $OUT/l2.log 2>&1 || exit 1
python3 $R/profiles/rocpd_summary.py $OUT/l2/run_results.db > $OUT/l2.txt || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_STREAMING_REQ_sum -d $OUT/l2calib -o run -- $R/profiles/fetch_calib > /dev/null 2> $OUT/l2calib.err || exit 1
python3 $R/profiles/rocpd_summary.py $OUT/l2calib/run_results.db > $OUT/l2calib.txt || exit 1
echo done
