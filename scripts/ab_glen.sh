# kernel time vs reference size (table in L2/MALL vs HBM)
for gl in 100000 400000 2000000; do
  for v in "PA_WALK_ROUNDS=1" "PA_WALK_ROUNDS=0"; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --genome-len $gl > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('glen $gl $v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms', d['index']['table_bytes']>>20, 'MiB')"
  done
done
