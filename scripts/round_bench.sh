# Round measurement: full bench line (CPU baseline + parity sample), rocprof kernel
# summary of the same command, and a FETCH_SIZE PMC pass for the traffic figure.
# usage: bash scripts/round_bench.sh <tag> [bench args...]
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/rb_$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/pmc.log 2>&1 || exit 1
echo done
