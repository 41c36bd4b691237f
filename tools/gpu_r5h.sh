#!/bin/bash
# LocalBA tests, then A/B: HEAD (base3) vs this tree; LDLT stamps
mkdir -p gpurun_out
rm -f gpurun_out/r5b_ba_ab.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_localba.py tests/test_shim.py > gpurun_out/r5h_tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5h_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base3 cur base3 cur base3 cur; do
  if [ $v = cur ]; then lib=; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 20 >> gpurun_out/r5b_ba_ab.txt 2>&1 || exit 1
  echo "^ $v" >> gpurun_out/r5b_ba_ab.txt
done
for v in base3 cur; do
  if [ $v = cur ]; then lib=; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib tools/kprof.sh kp5b_ba_$v tools/ba_time.py 10 > /dev/null 2>&1 || exit 1
done
timeout -k 10 60 python tools/ldlt_stamps.py 120 > gpurun_out/ldlt_stamps2.json 2>&1
