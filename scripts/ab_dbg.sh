# timing dissection of the fast kernel with the PA_STATS build (results invalid for modes > 0)
export PA_LIBRARY=$PWD/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/libpa_stats.so
for v in "PA_DBG_MODE=0" "PA_DBG_MODE=1" "PA_DBG_MODE=2" "PA_DBG_MODE=3" "PA_DBG_MODE=4" "PA_DBG_MODE=3 PA_WALK_ROUNDS=0" "PA_DBG_MODE=4 PA_WALK_ROUNDS=0"; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
