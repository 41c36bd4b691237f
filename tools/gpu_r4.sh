#!/bin/bash
# round-4 GPU pass: smoke + GPU tests, then the default bench (one JSON line -> gpurun_out/bench.json).
# Plain test failures (exit 1) still let the bench run; a crash, abort or time limit ends the call.
mkdir -p gpurun_out
bash tools/gpu_check.sh
trc=$?
if [ $trc -ne 0 ] && [ $trc -ne 1 ]; then exit $trc; fi
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"
tail -c 1500 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROF" ] && exit $trc
bash tools/prof_r4.sh || exit $?
exit $trc
