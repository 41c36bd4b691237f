#!/bin/bash
# Run smoke + GPU tests on the box; stop at the first crash/timeout (a plain
# assertion failure of smoke still lets the test suite run, for diagnosis).
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 ${GPU_TEST_TIMEOUT:-500} python -m pytest tests -m gpu -q ${PYTEST_ARGS:--x} --tb=short > gpurun_out/gpu_tests.log 2>&1
rc2=$?
echo "tests rc=$rc2"
tail -5 gpurun_out/gpu_tests.log
exit $rc2
