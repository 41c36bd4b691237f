#!/bin/bash
# Round-3 final evidence (GPU box): smoke + GPU suite, the default bench line, then rocprofv3
# (kernel stats of the bench, FETCH_SIZE / WRITE_SIZE passes, LocalBA and PnP kernel stats).
bash tools/gpu_check.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
OUT=gpurun_out/prof bash tools/profile.sh
