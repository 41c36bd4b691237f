#!/bin/bash
# LocalBA per-kernel mean durations (rocprofv3 --kernel-trace --stats on tools/ba_time.py) for the
# in-tree library and build_ab/$1, then ba_time alternating four rounds
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
V=$1
O=gpurun_out/bak_$V
mkdir -p $O
R=$PWD
for v in base $V; do
  lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$v -o ba --output-format csv -- python3 tools/ba_time.py 20 > /dev/null 2>&1 || exit 1
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1)
  echo "$v $(python3 tools/kstats_brief.py $f)"
done
for rep in 1 2 3 4; do
  for v in base $V; do
    lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/t_${v}_$rep.json || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/t_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
  done
done
