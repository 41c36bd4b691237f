#!/bin/bash
# LocalBA ba_time A/B, current library vs build_ab/head, 5 alternating runs of 40 calls
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5o
for rep in 1 2 3 4 5; do
  for v in base head; do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > gpurun_out/r5o/ba_${v}_$rep.json
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r5o/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
  done
done
