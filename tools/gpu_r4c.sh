#!/bin/bash
# round-4 iteration: full GPU suite first (diagnostics), then the A/B of build_ab variants, then bench+prof
mkdir -p gpurun_out
NO_PROF=1 PYTEST_ARGS="-q --timeout 120 --timeout-method thread" bash tools/gpu_r4.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab.sh || exit $?
bash tools/prof_r4.sh || exit $?
exit $rc
