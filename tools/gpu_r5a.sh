#!/bin/bash
# round-5 GPU pass: the full GPU suite, single-call matcher latency (+ kernel stats), the stereo
# rows-only floor (FETCH / WRITE passes of the probe build).  A failing step ends the call.
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r5_full_tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5_full_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/matcher_latency.py 50 > gpurun_out/r5_matcher_lat.json 2>&1 || exit 1
tools/kprof.sh kp_matcher tools/matcher_latency.py 20 > gpurun_out/kp_matcher.txt 2>&1 || exit 1
ORBX_LIB_OVERRIDE=$PWD/build_ab/rowsprobe/liborbx.so OUT=gpurun_out/tn_floor bash tools/traffic_now.sh > gpurun_out/tn_floor.txt 2>&1
