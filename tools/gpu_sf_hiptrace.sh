#!/bin/bash
# Host-side timeline of the drop-in stereo Frame: HIP API + kernel + memory-copy trace of frame_bench
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/sf_hip
mkdir -p $O
python tools/single_frame_prof.py make $O/frames.u8 8 || exit 1
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $O/trace -o sf -- shim/build/frame_bench $O/frames.u8 1241 376 8 60 20 2000 386.1448 718.856 > $O/out.json 2> $O/err.log || exit 1
tail -1 $O/out.json
rm -f $O/frames.u8
