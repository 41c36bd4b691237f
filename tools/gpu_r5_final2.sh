#!/bin/bash
# Round-5 close-out after the LocalBA call-level changes: full GPU suite, LocalBA kernel-trace +
# FETCH / WRITE passes (tools/ba_time.py), then the default bench line.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/fin2/ba
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/fin2/gputest.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/fin2/gputest.log; [ $rc -eq 0 ] || exit $rc
tail -2 gpurun_out/fin2/gputest.log
set -e
OUT=gpurun_out/fin2/ba
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/ba_time.py 10 > $OUT/trace.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/ba_time.py 10 > $OUT/fetch.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/ba_time.py 10 > $OUT/write.log 2>&1
echo "ba passes ok"
timeout -k 10 600 python bench.py > gpurun_out/fin2/bench.json 2> gpurun_out/fin2/bench.err
tail -c 600 gpurun_out/fin2/bench.json
