#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group per pass, no trace domains) of a
# short bench run; summarise locally with: python tools/traffic_now.py gpurun_out/tn
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/tn}
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 --profile-steps 0}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
echo "fetch ok"
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo "write ok"
