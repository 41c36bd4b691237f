#!/bin/bash
# LDLT variant A/B: LocalBA tests with the in-tree library, then the reduced-system LDLT alone
# (tools/ldlt_bench.py) and the config-4 call (tools/ba_time.py) alternating with build_ab/$1.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
V=$1
O=gpurun_out/ldlt_$V
mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_localba.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in base $V; do
    lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
    echo "$v ldlt $(ORBX_LIB_OVERRIDE=$lib timeout -k 10 60 python tools/ldlt_bench.py 60 120 | python3 -c 'import json,sys; print([round(json.loads(l)["ms"]*1e3,2) for l in sys.stdin])')" || exit 1
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json || exit 1
    echo "$v call $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4), d['iterations'], d['trials'])")"
  done
done
