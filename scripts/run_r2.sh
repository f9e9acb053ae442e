# counter pass (fabric lines + SQ shares per align kernel) of bench configs
set -o pipefail
mkdir -p gpurun_out/r2
for c in ${CONFIGS:-c2rc c2mix}; do
timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --profile-dir gpurun_out/r2/$c $BENCH_ARGS > gpurun_out/r2/$c.json 2> gpurun_out/r2/$c.err || { tail -5 gpurun_out/r2/$c.err; exit 1; }
python3 - $c <<'PY'
import json, sys
c = sys.argv[1]
d = json.load(open(f'gpurun_out/r2/{c}.json')); r = d['roofline']
print(c, round(d['value'] / 1e9, 3), 'G/s')
for k, v in r['kernels'].items():
    sq = v.get('sq_share_of_wave_cycles') or {}
    print(' ', k, round(v.get('ms_avg', 0), 3), 'ms', 'lines/read', round(v.get('lines_per_read', 0), 2), {a: round(b, 3) for a, b in sq.items()})
PY
done
