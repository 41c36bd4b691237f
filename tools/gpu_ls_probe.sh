#!/bin/bash
# k_ba_lin_schur phase stamps (probe build build_ab/lsprobe), three runs
set -e
mkdir -p gpurun_out
for r in 1 2 3; do ORBX_LIB_OVERRIDE=$PWD/build_ab/lsprobe/liborbx.so timeout -k 10 120 python tools/ls_probe.py | tee -a gpurun_out/ls_probe.txt; done
