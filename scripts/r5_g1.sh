set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r5a; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_reduce.py tests/test_gpu_parity.py::test_align_without_reference_file_fails_like_the_reference tests/test_bench_launch.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
PA_CLI_TIMING=1 timeout -k 10 700 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --profile-dir $OUT > $OUT/c5.json 2> $OUT/c5.err || { tail -20 $OUT/c5.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/c5.json')); r=d['roofline']
print('c5', round(d['value']/1e9,3), 'frac', r['frac'], r['traffic_basis'][:300])"
