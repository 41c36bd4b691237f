#!/bin/bash
# LocalBA host-side marks (library trace option), current library, 3 runs
set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r5t
for rep in 1 2 3; do timeout -k 10 200 python tools/ba_hostmarks.py 40 | tee gpurun_out/r5t/marks_$rep.json; done
