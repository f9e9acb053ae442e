#!/bin/bash
# Round-2 measurement on the GPU box: FETCH_SIZE calibration, C2 bench line
# (in-run traffic + CPU baseline), SQ counters of the C2 align pass, and the
# robustness line.  usage: bash scripts/r02_measure.sh <tag>
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/m_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/calib -o run -- $R/profiles/fetch_calib > $OUT/calib.json 2> $OUT/calib.err || exit 1
python3 $R/profiles/rocpd_summary.py $OUT/calib/run_results.db > $OUT/calib_pmc.txt || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $OUT/calib2 -o run -- $R/profiles/fetch_calib > /dev/null 2> $OUT/calib2.err && python3 $R/profiles/rocpd_summary.py $OUT/calib2/run_results.db > $OUT/calib_req.txt
echo calib done
cd $R
timeout -k 10 600 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 1
echo bench c2 done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d $OUT/sq_c2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/sq_c2.log 2>&1 || exit 1
python3 $R/profiles/rocpd_summary.py $OUT/sq_c2/run_results.db > $OUT/sq_c2.txt || exit 1
echo sq done
cd $R
timeout -k 10 600 python bench.py --config c2mix > $OUT/bench_c2mix.json 2> $OUT/bench_c2mix.err || exit 1
echo all done
