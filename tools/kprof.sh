#!/bin/bash
# Per-kernel stats of one python tool under rocprofv3 (GPU box):
#   tools/kprof.sh NAME tools/x.py [args...]
set -e
NAME=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$NAME
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/"$@" > $OUT.log 2>&1
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -20
