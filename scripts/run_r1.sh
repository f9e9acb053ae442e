# quick GPU check: parity of the no-seed paths + positions, then short benches
set -o pipefail
mkdir -p gpurun_out/r1
timeout -k 10 500 python -u -m pytest tests/test_gpu_positions.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r1/tests.log 2>&1 || { tail -30 gpurun_out/r1/tests.log; exit 1; }
tail -3 gpurun_out/r1/tests.log
for c in ${CONFIGS:-c2rc c2mix c2}; do
timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-traffic --no-e2e $BENCH_ARGS > gpurun_out/r1/$c.json 2> gpurun_out/r1/$c.err || { tail -5 gpurun_out/r1/$c.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r1/$c.json')); r=d['roofline']
print('$c', round(d['value']/1e9,3), {k: round(v['ms_avg'],3) for k, v in r['kernels'].items()}, round(d['index']['build_s'],3), (d.get('parity_sample') or {}).get('bit_exact'))"
done
