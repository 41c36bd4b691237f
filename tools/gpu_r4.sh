#!/bin/bash
# round-4 GPU pass: smoke + GPU tests, then the default bench (one JSON line -> gpurun_out/bench.json).
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"
tail -c 1500 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_PROF" ] && exit 0
bash tools/prof_r4.sh
