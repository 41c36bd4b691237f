#!/bin/bash
# tools/ba_time.py (config 4) for the in-tree library and each build_ab variant, alternating
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/bav
mkdir -p $O
R=$PWD
for rep in 1 2 3; do
  for v in base "$@"; do
    lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/${v}_$rep.json || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4), d['iterations'], d['trials'])")"
  done
done
