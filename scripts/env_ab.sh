#!/bin/bash
# Bench lines of one config under several environment settings (A/B of the
# library's runtime knobs), build stage times included (PA_CLI_TIMING=1):
#   CFG=c5 ENVS="base PA_BUILD_RUN=4 PA_BLOOM_HBM=0,PA_BUILD_RUN=8" STEPS=5 bash scripts/env_ab.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/env_$1
mkdir -p $OUT
cd $R
i=0
for v in $ENVS; do
  i=$((i+1))
  e=""; [ "$v" != base ] && e=${v//,/ }
  env PA_CLI_TIMING=1 $e timeout -k 10 ${LIMIT:-400} python bench.py --config $CFG --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-e2e --no-traffic > $OUT/$i.json 2> $OUT/$i.err || { tail -5 $OUT/$i.err; exit 1; }
  python3 -c "
import json, re
d=json.load(open('$OUT/$i.json')); r=d['roofline']; ix=d['index']
err=open('$OUT/$i.err').read()
st=re.findall(r'(insert \+ sets|nb: first occurrences|nb: copies|tile classes|repeats \+ walk blocks) ([0-9.]+)', err)
print('$CFG $v', round(d['value']/1e6,1), 'Mreads/s, pass', round(r['algorithmic']['survey_8d']['pass_ms'],3), 'ms, index', round(ix['build_s'],2), 's', st)"
done
