# phase dissection (stats build) on a MALL-resident reference: compute cost per phase
export PA_LIBRARY=$PWD/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/libpa_stats.so
for gl in 100000 2000000; do
for v in "PA_DBG_MODE=2" "PA_DBG_MODE=3" "PA_DBG_MODE=4" "PA_DBG_MODE=0"; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --genome-len $gl > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('glen $gl $v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
done
