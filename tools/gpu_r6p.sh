#!/bin/bash
# Round-6 call J: LocalBA with phase 2's outlier marking + structure queued (see commit)
# 1's readback (one host round trip fewer per call): LocalBA / pipeline / shim GPU tests, then
# tools/ba_time.py alternating base and the seqsum build, four rounds.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r6p
mkdir -p $O
R=$PWD
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_localba.py tests/test_pipeline.py tests/test_shim.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3 4; do
  for v in base seqsum; do
    lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4), d['iterations'], d['trials'])")"
  done
done
echo done
