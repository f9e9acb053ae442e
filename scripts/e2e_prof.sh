#!/bin/bash
# End-to-end dumpalign on the C2 files: the e2e JSON line, then a rocprofv3
# kernel trace of the CLI command itself (where the device time goes).
# usage (GPU box): bash scripts/e2e_prof.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/e2e_$1
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u scripts/e2e_cli.py --keep --dir /tmp/pa_e2e > $OUT/e2e.json 2> $OUT/e2e.err || exit 1
echo e2e done
cd /tmp && export TMPDIR=/tmp
PA_FAST_EXIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $R/bioinformatics-project-for-shotgun-metagenomics-pseudo-alignment-shotgun-_amd/main.py -t dumpalign -g /tmp/pa_e2e/c2.fa -k 31 --reads /tmp/pa_e2e/c2.fq > $OUT/trace.log 2>&1 || exit 1
echo trace done
