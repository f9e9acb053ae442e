# GPU parity tests + C2 bench variants + lane statistics
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gputest.log 2>&1; tail -3 gpurun_out/gputest.log
for v in "PA_NO_LANE=0" "PA_NO_LANE=1" ${EXTRA_VARIANTS}; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('${v##*/}', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
PA_LIBRARY=$PWD/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/libpa_stats.so timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline $BENCH_ARGS 2>&1 | grep pa_stats | tail -1
