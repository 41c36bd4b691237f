#!/bin/bash
# A/B timing of library variants (build_ab/<v>/liborbx.so): bench.py stage timers (extraction +
# stereo) and tools/ba_time.py (LocalBA config 4, one problem) per variant, base first.
for v in base $(ls build_ab); do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms_per_step"])')"
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 20 > gpurun_out/ab_ba_$v.log 2>&1 || exit 1
  echo "$v ba $(tail -1 gpurun_out/ab_ba_$v.log)"
done
