#!/bin/bash
# full GPU suite after the LDLT look-ahead change, then the LocalBA A/B against the previous commit
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r5d_tests.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r5d_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5b.sh
