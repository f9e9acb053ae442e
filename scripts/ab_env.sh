set -e
for v in "PA_WALK_ROUNDS=2" "PA_WALK_ROUNDS=1" "PA_WALK_ROUNDS=0" "PA_CAP_MULT=4 PA_WALK_ROUNDS=2" "PA_CAP_MULT=4 PA_WALK_ROUNDS=1" "PA_CAP_MULT=4 PA_WALK_ROUNDS=0"; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
