# env-knob A/B of the C2 bench (VARIANTS="A=1 B=2,C=3 ..." -- comma joins settings of one variant)
for v in $VARIANTS; do
  env ${v//,/ } timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
