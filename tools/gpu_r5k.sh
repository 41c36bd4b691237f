#!/bin/bash
# resize+blur fusion: extraction/stereo parity tests, then stage timers of the current library
# against build_ab/* (bench.py stage timers, 3 alternating runs each)
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5k
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_stereo.py > gpurun_out/r5k/tests.log 2>&1 || { tail -30 gpurun_out/r5k/tests.log; exit 1; }
tail -2 gpurun_out/r5k/tests.log
for rep in 1 2 3; do
for v in base $(ls build_ab); do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --single-frames 0 --track-steps 0 > gpurun_out/r5k/ab_${v}_$rep.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r5k/ab_${v}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms_per_step"])')"
done
done
