#!/bin/bash
# rocprofv3 evidence (run on the GPU box):
#   pass 1: --kernel-trace --stats of bench.py  -> per-kernel average durations
#   pass 2: --pmc FETCH_SIZE (own pass)         -> HBM read bytes per dispatch
#   pass 3: --pmc WRITE_SIZE (own pass)         -> HBM write bytes per dispatch
#   pass 4/5: --kernel-trace --stats of the LocalBA and PnP timing tools
# Counters are collected in passes without any trace domain (gpurun rule).
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/prof}
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --inflight 1 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
echo "fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo "write ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/localba -o run --output-format csv -- python3 tools/ba_time.py 10 > $OUT/localba.log 2>&1
echo "localba ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pnp -o run --output-format csv -- python3 tools/pnp_time.py > $OUT/pnp.log 2>&1
echo "pnp ok"
find $OUT -name "*stats.csv" | head -20
