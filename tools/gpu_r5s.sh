#!/bin/bash
# LocalBA lambda init + LM init in one launch (k_ba_lm_start): LocalBA/pipeline/shim GPU tests, ba_time A/B against
# build_ab/head (5 alternating runs of 40 calls), timeline of one call
set -e
cd /tmp && export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5s
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py tests/test_pipeline.py tests/test_shim.py > gpurun_out/r5s/tests.log 2>&1 || { tail -30 gpurun_out/r5s/tests.log; exit 1; }
tail -2 gpurun_out/r5s/tests.log
for rep in 1 2 3 4 5; do
  for v in base head; do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > gpurun_out/r5s/ba_${v}_$rep.json
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r5s/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r5s/trace -o trace --output-format csv -- python3 tools/ba_time.py 3 > gpurun_out/r5s/trace.log 2>&1
python tools/ba_timeline.py gpurun_out/r5s/trace > gpurun_out/r5s/timeline.txt
tail -1 gpurun_out/r5s/timeline.txt
