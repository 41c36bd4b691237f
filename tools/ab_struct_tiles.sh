#!/bin/bash
# LocalBA structure-build tile size A/B: tests, per-kernel stats of k_ba_struct_*, ba_time for the current library and build_ab/sv4, sv2
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/ab_sv; mkdir -p $O
for v in base sv4 sv2; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py > $O/tests_$v.log 2>&1 || { tail -20 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/ba_time.py 10 > $O/prof_$v.log 2>&1
  python3 - "$v" <<'PY'
import csv,glob,sys
f=glob.glob('gpurun_out/ab_sv/prof_%s/**/*kernel_stats.csv'%sys.argv[1],recursive=True)[0]
print(sys.argv[1], {r['Name'].split('(')[0].replace('orbx::',''):round(float(r['AverageNs'])/1e3,2) for r in csv.DictReader(open(f)) if 'struct' in r['Name']})
PY
done
for rep in 1 2 3; do for v in base sv4 sv2; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json
  echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
done; done
