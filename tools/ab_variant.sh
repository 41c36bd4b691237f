#!/bin/bash
# A/B of library variants on the GPU box: the extraction / stereo parity tests run WITH each
# build_ab/<variant>/liborbx.so, then bench.py stage timers alternating the default library ("base")
# with the variants, three rounds.   usage: bash tools/ab_variant.sh OUTDIR VARIANT...
O=$1; shift
mkdir -p $O
for v in "$@"; do
  ORBX_LIB_OVERRIDE=$PWD/build_ab/$v/liborbx.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_stereo.py > $O/tests_$v.log 2>&1 || { echo "$v: tests failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
for rep in 1 2 3; do
  for v in base "$@"; do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > $O/${v}_$rep.log 2>&1 || { echo "$v bench failed"; tail -5 $O/${v}_$rep.log; exit 1; }
    echo "$v $(tail -1 $O/${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["stage_ms_per_step"])')"
  done
done
