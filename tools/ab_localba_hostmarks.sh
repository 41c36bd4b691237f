#!/bin/bash
# LocalBA host marks (library trace option) for the current library and each build_ab variant,
# alternating, three rounds, then the GPU tests of the current library.  usage: bash tools/ab_localba_hostmarks.sh [outdir]
set -e
O=${1:-gpurun_out/ab_hostmarks}; mkdir -p $O
for rep in 1 2 3; do for v in base $(ls build_ab 2>/dev/null); do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 python tools/ba_hostmarks.py 40 > $O/marks_${v}_$rep.json
  echo "$v $(cat $O/marks_${v}_$rep.json)"
done; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py tests/test_shim.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
