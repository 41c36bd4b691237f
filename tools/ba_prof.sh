#!/bin/bash
# LocalBA per-kernel times (GPU box): tools/ba_prof.sh [calls]
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/bap
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ba_time.py ${1:-10} > $OUT.log 2>&1
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -20
