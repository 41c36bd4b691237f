#!/bin/bash
# LocalBA write-back change: LocalBA + shim GPU tests, ba_time A/B against build_ab/head (3 alternating
# runs), and a kernel + copy timeline of one call
set -e
cd /tmp && export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5n
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py tests/test_pipeline.py > gpurun_out/r5n/tests.log 2>&1 || { tail -30 gpurun_out/r5n/tests.log; exit 1; }
tail -2 gpurun_out/r5n/tests.log
for rep in 1 2 3; do
  for v in base head; do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 30 > gpurun_out/r5n/ba_${v}_$rep.json
    echo "$v $(cat gpurun_out/r5n/ba_${v}_$rep.json)"
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r5n/trace -o trace --output-format csv -- python3 tools/ba_time.py 3 > gpurun_out/r5n/trace.log 2>&1
python tools/ba_timeline.py gpurun_out/r5n/trace > gpurun_out/r5n/timeline.txt
tail -4 gpurun_out/r5n/timeline.txt
