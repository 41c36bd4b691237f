#!/bin/bash
# Kernel-trace of the default (4 batches in flight) headline loop: do kernels of different slots'
# streams overlap?  Output gpurun_out/ovl/run_kernel_trace.csv; analyse with tools/overlap.py.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ovl
timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/ovl -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --profile-steps 0 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > gpurun_out/ovl/log 2>&1
