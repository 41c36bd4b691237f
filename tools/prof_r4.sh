#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box after a build):
#   trace : --kernel-trace --stats of a short bench run      -> per-stage ms per step
#   fetch / write : --pmc FETCH_SIZE / WRITE_SIZE (own passes) -> HBM bytes per stage event
#   ba_* : the same three passes over tools/ba_time.py        -> LocalBA bytes per LM iteration
# Counters run in passes without trace domains (gpurun rule); each pass under its own time limit.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/prof}
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --inflight 1 --profile-steps 5 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0}
mkdir -p $OUT $OUT/ba
set -e
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
echo "trace ok"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
echo "fetch ok"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo "write ok"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/ba/trace -o run --output-format csv -- python3 tools/ba_time.py 10 > $OUT/ba/trace.log 2>&1
echo "ba trace ok"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/ba/fetch -o run --output-format csv -- python3 tools/ba_time.py 10 > $OUT/ba/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/ba/write -o run --output-format csv -- python3 tools/ba_time.py 10 > $OUT/ba/write.log 2>&1
echo "ba pmc ok"
find $OUT -name "*stats.csv" -o -name "*counter_collection.csv" | head -20
