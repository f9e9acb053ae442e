# reads-per-step A/B (main build) and memory dissection (stats build; results invalid for modes > 0)
for v in "PA_READS_PER_STEP=1" "PA_READS_PER_STEP=2" "PA_READS_PER_STEP=4" "PA_READS_PER_STEP=2 PA_WALK_ROUNDS=1" "PA_READS_PER_STEP=1 PA_WALK_ROUNDS=1"; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
done
export PA_LIBRARY=$PWD/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/libpa_stats.so
for v in "PA_DBG_MODE=0 PA_READS_PER_STEP=1" "PA_DBG_MODE=5 PA_READS_PER_STEP=1 PA_WALK_ROUNDS=0" "PA_DBG_MODE=6 PA_READS_PER_STEP=1 PA_WALK_ROUNDS=0" "PA_DBG_MODE=0 PA_READS_PER_STEP=1 PA_WALK_ROUNDS=0" "PA_DBG_MODE=3 PA_READS_PER_STEP=1 PA_WALK_ROUNDS=0" "PA_DBG_MODE=3 PA_READS_PER_STEP=2 PA_WALK_ROUNDS=0" "PA_DBG_MODE=3 PA_READS_PER_STEP=1 PA_WALK_ROUNDS=1"  "PA_DBG_MODE=3 PA_READS_PER_STEP=2 PA_WALK_ROUNDS=1"; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],2), 'ms')"
  grep pa_stats gpurun_out/ab.err | tail -1
done
