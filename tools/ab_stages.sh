#!/bin/bash
# Extraction A/B on the GPU box: the extraction / stereo parity tests with the current library, then
# bench.py stage timers (ms per 256-frame step, 4 in flight) alternating the current library ("base")
# with every build_ab/<variant>/liborbx.so, three rounds.   usage: bash tools/ab_stages.sh [outdir]
set -e
O=${1:-gpurun_out/ab_stages}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_stereo.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in base $(ls build_ab 2>/dev/null); do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > $O/${v}_$rep.log 2>&1
    echo "$v $(tail -1 $O/${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["stage_ms_per_step"])')"
  done
done
