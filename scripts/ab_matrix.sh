# bench configs x library variants (no CPU baseline): CONFIGS="c2 c3" LIBS="libpa.so libpa_x.so"
L=$PWD/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
for c in ${CONFIGS:-c2}; do
  for lib in ${LIBS:-libpa.so}; do
    PA_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$c $lib', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],3), 'ms')"
  done
done
