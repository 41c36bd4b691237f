#!/bin/bash
# LocalBA A/B on the GPU box: the LocalBA / pipeline / shim GPU tests with the current library, then
# tools/ba_time.py (40 calls; mean and median ms per call) alternating the current library ("base")
# with every build_ab/<variant>/liborbx.so, five rounds, and a kernel + memory-copy timeline of one
# call (tools/ba_timeline.py).   usage: bash tools/ab_localba.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=${1:-gpurun_out/ab_localba}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py tests/test_pipeline.py tests/test_shim.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3 4 5; do
  for v in base $(ls build_ab 2>/dev/null); do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json
    echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o trace --output-format csv -- python3 tools/ba_time.py 3 > $O/trace.log 2>&1
python tools/ba_timeline.py $O/trace > $O/timeline.txt
tail -1 $O/timeline.txt
