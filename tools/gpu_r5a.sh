#!/bin/bash
# Round-5 GPU pass: LocalBA A/B (HEAD~ library vs this tree), the full GPU suite, single-call
# matcher latency (+ kernel trace), the stereo row-floor traffic probe, LDLT stamps, v_rcp_f64.
mkdir -p gpurun_out
for v in base cur pv1 pv2 nr1 up64 base cur pv1 pv2 nr1 up64; do
  if [ $v = cur ]; then lib=; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 20 >> gpurun_out/r5_ba_ab.txt 2>&1 || exit 1
  echo "^ $v" >> gpurun_out/r5_ba_ab.txt
done
for v in base cur pv1 pv2 nr1 up64; do
  if [ $v = cur ]; then lib=; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib tools/kprof.sh kp_ba_$v tools/ba_time.py 10 > gpurun_out/kp_ba_$v.txt 2>&1 || exit 1
done
timeout -k 10 60 python tools/ldlt_stamps.py 120 > gpurun_out/ldlt_stamps.json 2>&1
timeout -k 10 60 tools/micro/rcp_bench > gpurun_out/rcp_bench.json 2>&1
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r5_full_tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5_full_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/matcher_latency.py 50 > gpurun_out/r5_matcher_lat.json 2>&1 || exit 1
tools/kprof.sh kp_matcher tools/matcher_latency.py 20 > gpurun_out/kp_matcher.txt 2>&1 || exit 1
ORBX_LIB_OVERRIDE=$PWD/build_ab/rowsprobe/liborbx.so OUT=gpurun_out/tn_floor bash tools/traffic_now.sh > gpurun_out/tn_floor.txt 2>&1
