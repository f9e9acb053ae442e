# timing dissection of the lane kernel (PA_DISSECT build; results invalid for modes > 0):
# 13 stop after the packing, 14 one seed round, 10 after the seeds, 11 after the walk, 12 no second walk, 0 full
L=$PWD/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd
for c in ${CONFIGS:-c2}; do
  for m in ${MODES:-13 10 11 12 0}; do
    PA_LIBRARY=$L/libpa_dissect.so PA_DBG_MODE=$m timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-traffic --no-e2e > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$c mode $m', round(d['value']/1e6,1), 'Mreads/s', round(d['roofline']['kernel_ms'],3), 'ms')"
  done
done
