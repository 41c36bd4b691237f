mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_golden.py tests/test_shim.py tests/test_tracking.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t7.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t7.log
exit $rc
