#!/bin/bash
# round-4 iteration: tracking + stereo tests alone, A/B of build_ab variants, then the full pass
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_tracking.py tests/test_gpu_stereo.py -q --timeout 120 --timeout-method thread > gpurun_out/trk.log 2>&1
rc=$?; echo "trk+stereo rc=$rc"; tail -15 gpurun_out/trk.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/ab.sh || exit $?
NO_PROF=${NO_PROF:-} PYTEST_ARGS="-q --timeout 120 --timeout-method thread" bash tools/gpu_r4.sh
