# bench C2 with library variants
L=$PWD/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
for lib in libpa.so $LIBS; do
  PA_LIBRARY=$L/$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
