# bench lines for the other configs (parity sample on, short runs)
for c in c3 c3raw c1; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 > gpurun_out/cfg_$c.json 2> gpurun_out/cfg_$c.err || { tail -5 gpurun_out/cfg_$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/cfg_$c.json')); print('$c', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms', d['roofline']['frac'], d.get('parity_sample'))"
done
timeout -k 10 300 python bench.py --config c2 --genome-len 200000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cfg_g500.json 2>&1
