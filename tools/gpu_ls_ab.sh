#!/bin/bash
# k_ba_lin_schur change: probe stamps (build_ab/lsprobe = the change + stamps), LocalBA tests, kernel A/B vs build_ab/head
set -e
for r in 1 2; do ORBX_LIB_OVERRIDE=$PWD/build_ab/lsprobe/liborbx.so timeout -k 10 120 python tools/ls_probe.py; done
mv build_ab/lsprobe /tmp/lsprobe_keep
bash tools/ab_localba_kernels.sh gpurun_out/ab_lscopy
