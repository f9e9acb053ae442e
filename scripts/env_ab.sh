#!/bin/bash
# Bench lines of one config under several environment settings (A/B of the
# library's runtime knobs), build stage times included (PA_CLI_TIMING=1):
#   CFG=c5 ENVS="base PA_BUILD_RUN=4 PA_BLOOM_HBM=0,PA_BUILD_RUN=8" STEPS=5 bash scripts/env_ab.sh <tag>
# (CPU=1: with the CPU baseline and its bit-exact oracle sample; the job
# counters' hash is printed either way: equal across settings = same results)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/env_$1
mkdir -p $OUT
cd $R
i=0
for v in $ENVS; do
  i=$((i+1))
  e=""; [ "$v" != base ] && e=${v//,/ }
  env PA_CLI_TIMING=1 $e timeout -k 10 ${LIMIT:-400} python bench.py --config $CFG --steps ${STEPS:-10} --warmup 2 $([ "$CPU" = 1 ] || echo --no-cpu-baseline) --no-e2e --no-traffic > $OUT/$i.json 2> $OUT/$i.err || { tail -5 $OUT/$i.err; exit 1; }
  python3 -c "
import json, re
d=json.load(open('$OUT/$i.json')); r=d['roofline']; ix=d['index']
err=open('$OUT/$i.err').read()
st=re.findall(r'(insert \+ sets|nb: first occurrences|nb: copies|tile classes|repeats \+ walk blocks) ([0-9.]+)', err)
ks={k: round(v['ms_avg'], 3) for k, v in r.get('kernels', {}).items()} or r['per_rank'][0]['kernels_ms']
ps=d.get('parity_sample') or {}
print('$CFG $v', round(d['value']/1e6,1), 'Mreads/s, ms', round(d['ms_per_step'],3), 'index', round(ix['build_s'],2), 's', st,
      'kernels', {k: round(v, 3) for k, v in ks.items() if v > 0.02}, 'job', d['job_counters']['sha256'][:12],
      'job s', round(d['job']['job_s'], 4), 'job pass ms', round(d['job']['align_pass_s'] * 1e3, 2),
      'parity', ps.get('bit_exact'), ps.get('reads'))"
done
