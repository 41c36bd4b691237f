#!/bin/bash
# round-3 GPU pass: smoke + GPU tests, then the A/B of build_ab variants, then the full bench.
bash tools/gpu_check.sh || exit $?
bash tools/ab.sh || exit $?
timeout -k 10 500 python bench.py ${BENCH_ARGS:---cpu-baseline-seconds 5} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -c 3000 gpurun_out/bench.log
exit $rc
