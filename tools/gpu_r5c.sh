#!/bin/bash
# stereo row floor (probe library), the Sim3 single-run change under the projection/shim tests, matcher latency
mkdir -p gpurun_out
ORBX_LIB_OVERRIDE=$PWD/build_ab/rowsprobe/liborbx.so timeout -k 10 200 python tools/stereo_floor.py 3 > gpurun_out/r5_stereo_floor.json 2>&1 || exit 1
ORBX_LIB_OVERRIDE=$PWD/build_ab/rowsprobe/liborbx.so OUT=gpurun_out/tn_floor2 bash tools/traffic_now.sh > gpurun_out/tn_floor2.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_projection.py tests/test_shim.py > gpurun_out/r5c_tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/matcher_latency.py 50 > gpurun_out/r5_matcher_lat2.json 2>&1 || exit 1
