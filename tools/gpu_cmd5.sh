mkdir -p gpurun_out
ORBX_LIB_OVERRIDE=$PWD/build_ab/fprobe/liborbx.so timeout -k 10 200 python tools/fast_probe.py > gpurun_out/fast_probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/fast_probe.log
timeout -k 10 300 python -u -m pytest tests/test_tracking.py tests/test_gpu_stereo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/t5.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --single-frames 0 --track-steps 5 > gpurun_out/bench5.log 2>&1; echo "bench rc=$?"; tail -c 1500 gpurun_out/bench5.log
