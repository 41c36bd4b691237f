#!/bin/bash
# LocalBA: GPU tests (LocalBA, pipeline, shim, tracking), host marks, ba_time A/B vs build_ab/head
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5u
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py tests/test_pipeline.py tests/test_shim.py tests/test_tracking.py > gpurun_out/r5u/tests.log 2>&1 || { tail -30 gpurun_out/r5u/tests.log; exit 1; }
tail -1 gpurun_out/r5u/tests.log
timeout -k 10 200 python tools/ba_hostmarks.py 40 | tee gpurun_out/r5u/marks.json
for rep in 1 2 3 4 5; do
  for v in base head; do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > gpurun_out/r5u/ba_${v}_$rep.json
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r5u/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
  done
done
