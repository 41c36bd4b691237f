#!/bin/bash
# k_stereo_prep phase cost on the single stereo frame (build_ab/stopN: one-off builds of a temporary
# patch that returned early from k_stereo_prep; the patch is not kept): kernel durations with the kernel cut after
# the sort (stop1), after the sorted writes + octave starts (stop2), after the row table (stop3)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/prep_probe
mkdir -p $O
python tools/single_frame_prof.py make $O/frames.u8 8 || exit 1
for v in base stop1 stop2 stop3; do
  lp=""; [ $v = base ] || lp=$PWD/build_ab/$v
  LD_LIBRARY_PATH=$lp timeout -k 10 180 rocprofv3 --kernel-trace -d $O/$v -o sf -- shim/build/frame_bench $O/frames.u8 1241 376 8 100 20 2000 386.1448 718.856 > /dev/null 2>&1 || exit 1
  echo "$v $(python tools/single_frame_prof.py parse $O/$v | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["per_kernel_us_median"].get("orbx::k_stereo_prep"))')"
done
rm -f $O/frames.u8
