#!/bin/bash
# LocalBA A/B with per-kernel times: LocalBA GPU tests and rocprofv3 kernel stats per library (current
# = base, then build_ab/*), then ba_time.py (40 calls) alternating them, three rounds.
#   usage: bash tools/ab_localba_kernels.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=${1:-gpurun_out/ab_lbk}; mkdir -p $O
V="base $(ls build_ab 2>/dev/null)"
for v in $V; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py > $O/tests_$v.log 2>&1 || { tail -20 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 tools/ba_time.py 10 > $O/prof_$v.log 2>&1
  python3 - "$O" "$v" <<'PY'
import csv,glob,sys
f=glob.glob('%s/prof_%s/**/*kernel_stats.csv'%(sys.argv[1],sys.argv[2]),recursive=True)[0]
rows=[r for r in csv.DictReader(open(f))]
tot=sum(float(r['TotalDurationNs']) for r in rows)/1e3
print(sys.argv[2], 'total_us', round(tot,1), {r['Name'].split('(')[0].replace('orbx::','').replace('void ',''):round(float(r['AverageNs'])/1e3,2) for r in rows if float(r['TotalDurationNs'])>2e5})
PY
done
for rep in 1 2 3; do for v in $V; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json
  echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4))")"
done; done
