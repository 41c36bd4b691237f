#!/bin/bash
# smoke + GPU tests, then (only if both pass) a bench run.
bash tools/gpu_check.sh || exit $?
timeout -k 10 400 python bench.py ${BENCH_ARGS:---cpu-baseline-seconds 5} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -1 gpurun_out/bench.log
exit $rc
