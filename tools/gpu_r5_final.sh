#!/bin/bash
# Round-5 evidence: full GPU suite, rocprofv3 kernel-trace + FETCH/WRITE passes (bench and LocalBA),
# SQ counter passes, then the default bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/r05_gputest.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/r05_gputest.log; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/prof5 bash tools/prof_r4.sh > gpurun_out/prof5.log 2>&1 || exit 1
OUT=gpurun_out/pmc5 bash tools/pmc_kernel.sh > gpurun_out/pmc5.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r05_bench_pre.json 2> gpurun_out/r05_bench_pre.err || exit 1
