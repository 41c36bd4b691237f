#!/bin/bash
# k_ba_pairs block -> XCD mapping A/B: time, kernel stats and FETCH bytes (this tree vs pxcd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -f gpurun_out/r5b_ba_ab.txt
for v in cur pxcd cur pxcd cur pxcd; do
  if [ $v = cur ]; then lib=; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 20 >> gpurun_out/r5b_ba_ab.txt 2>&1 || exit 1
  echo "^ $v" >> gpurun_out/r5b_ba_ab.txt
done
for v in cur pxcd; do
  if [ $v = cur ]; then lib=; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib tools/kprof.sh kp5b_ba_$v tools/ba_time.py 10 > /dev/null 2>&1 || exit 1
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/bafetch_$v -o run --output-format csv -- python3 tools/ba_time.py 10 > gpurun_out/bafetch_$v.log 2>&1 || exit 1
done
ORBX_LIB_OVERRIDE=$PWD/build_ab/pxcd/liborbx.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py > gpurun_out/r5g_tests.log 2>&1; echo rc=$? >> gpurun_out/r5g_tests.log
