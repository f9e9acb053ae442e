# bench configs x environment variants (no CPU baseline): CONFIGS="c2 c4" VARIANTS="PA_BLOOM_MB=0 PA_BLOOM_MB=128"
for c in ${CONFIGS:-c2}; do
  for v in ${VARIANTS:-X=0}; do
    env $v timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$c $v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],3), 'ms', 'build', round(d['index']['build_s'],2))"
  done
done
