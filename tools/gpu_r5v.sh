#!/bin/bash
# k_ba_pairs two positions per step: LocalBA GPU tests, ba_time A/B vs build_ab/head (HEAD), kernel stats of both
set -e
cd /tmp && export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5v
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py > gpurun_out/r5v/tests.log 2>&1 || { tail -30 gpurun_out/r5v/tests.log; exit 1; }
tail -1 gpurun_out/r5v/tests.log
for rep in 1 2 3 4; do
  for v in base head; do
    if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > gpurun_out/r5v/ba_${v}_$rep.json
    echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/r5v/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
  done
done
for v in base head; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5v/prof_$v -o run --output-format csv -- python3 tools/ba_time.py 10 > gpurun_out/r5v/prof_$v.log 2>&1
  echo "== $v"; python3 - "$v" <<'PY'
import csv,glob,sys
f=glob.glob('gpurun_out/r5v/prof_%s/**/*kernel_stats.csv'%sys.argv[1],recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('k_ba_pairs','ldlt_pan','lin_schur','errors_ctl','k_ba_update','schur_fin')): print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2))
PY
done
