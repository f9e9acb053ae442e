# memory-pipeline counters of the align pass (one rocprofv3 pass per group)
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_ta
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1
i=0
for grp in "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" "TD_BUSY_avr GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" "TCC_REQ_sum TCC_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
echo done
