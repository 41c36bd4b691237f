#!/bin/bash
# Drop-in stereo Frame: one orbx_frame_stereo call (fused, default) against the reference's two
# extraction threads + ComputeStereoMatches (threads): stereo / shim GPU tests, frame_bench A/B
# alternating three rounds, then a kernel trace of the fused path.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/sf_ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stereo.py tests/test_shim.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
python tools/single_frame_prof.py make $O/frames.u8 8 || exit 1
for rep in 1 2 3; do
  for v in fused threads; do
    m=""; [ $v = fused ] || m=threads
    echo "$v $(timeout -k 10 120 shim/build/frame_bench $O/frames.u8 1241 376 8 300 20 2000 386.1448 718.856 $m | tail -1)" || exit 1
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/trace -o sf -- shim/build/frame_bench $O/frames.u8 1241 376 8 200 20 2000 386.1448 718.856 > $O/traced.json 2> $O/traced.err || exit 1
python tools/single_frame_prof.py parse $O/trace
rm -f $O/frames.u8
