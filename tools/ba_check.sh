mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_localba.py tests/test_shim.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ba_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ba_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/ba_time.py 20 && timeout -k 10 120 python tools/ba_time.py 20 && bash tools/ba_prof.sh 20
