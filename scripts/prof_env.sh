# rocprof kernel times for env variants (VARIANTS as in ab_env.sh)
cd /tmp && export TMPDIR=/tmp
i=0
for v in $VARIANTS; do
  i=$((i+1))
  env ${v//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/profv/$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $GRAFT_REPO_ROOT/gpurun_out/profv_$i.log 2>&1 || exit 1
  echo "$i $v" >> $GRAFT_REPO_ROOT/gpurun_out/profv/index.txt
done
