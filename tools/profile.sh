#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box):
#   pass 1: --kernel-trace --stats          -> per-kernel average durations
#   pass 2: --pmc FETCH_SIZE (own pass)     -> HBM read bytes per dispatch
#   pass 3: --pmc WRITE_SIZE (own pass)     -> HBM write bytes per dispatch
# Counters are collected in passes without any trace domain (gpurun rule).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/prof}
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo "write ok"
find $OUT -name "*.csv" | head -20
