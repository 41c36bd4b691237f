#!/bin/bash
# Build a liborbx.so variant into build_ab/NAME/ (objects in csrc/build_v_NAME):
#   tools/build_variant.sh NAME "-DORBX_FAST_PROBE"
set -e
NAME=$1; shift
make -s -j8 -C orb_slam2_commit_amd/csrc OBJDIR=build_v_$NAME OUT=../../build_ab/$NAME/liborbx.so EXTRA="$*"
