#!/bin/bash
# LocalBA call timeline: kernel + memory-copy trace of tools/ba_time.py (3 calls), and the host wall
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/r5j
cd $R
timeout -k 10 120 python tools/ba_time.py 20 > gpurun_out/r5j/wall.json
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/r5j/trace -o trace --output-format csv -- python3 tools/ba_time.py 3 > gpurun_out/r5j/trace.log 2>&1
python tools/ba_timeline.py gpurun_out/r5j/trace > gpurun_out/r5j/timeline.txt
tail -3 gpurun_out/r5j/timeline.txt; cat gpurun_out/r5j/wall.json
