# GPU parity tests + C2 bench variants
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gputest.log 2>&1; tail -3 gpurun_out/gputest.log
for v in "PA_WALK_ROUNDS=1" "PA_CAP_MULT=4" "PA_CAP_MULT=3" ${EXTRA_VARIANTS}; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('${v##*/}', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms', d['index'])"
done
