#!/bin/bash
# Drop-in single stereo frame: frame_bench timing alone, then a rocprofv3 kernel trace of the same run.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/sf
mkdir -p $O
python tools/single_frame_prof.py make $O/frames.u8 8 || exit 1
timeout -k 10 120 shim/build/frame_bench $O/frames.u8 1241 376 8 200 20 2000 386.1448 718.856 > $O/plain.json || exit 1
tail -1 $O/plain.json
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/trace -o sf -- shim/build/frame_bench $O/frames.u8 1241 376 8 200 20 2000 386.1448 718.856 > $O/traced.json 2> $O/traced.err || exit 1
tail -1 $O/traced.json
python tools/single_frame_prof.py parse $O/trace
rm -f $O/frames.u8
