#!/bin/bash
# per-level durations of the resize/blur kernels: current library and build_ab variants
set -e
cd /tmp && export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5l
for v in base $(ls build_ab); do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/build_ab/$v/liborbx.so; fi
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5l/$v -o run -- python3 bench.py --steps 4 --warmup 1 --inflight 1 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --single-frames 0 --track-steps 0 > gpurun_out/r5l/$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/kgrid_stats.py gpurun_out/r5l/$v k_resize k_blur
done
