#!/bin/bash
# Drop-in stereo Frame with the in-tree library (base) against build_ab/$1: stereo / shim / extract
# tests with base, then frame_bench alternating three rounds and a kernel trace of each.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
V=$1
O=gpurun_out/sf_$V
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_shim.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
python tools/single_frame_prof.py make $O/frames.u8 8 || exit 1
for rep in 1 2 3; do
  for v in base $V; do
    lp=""; [ $v = base ] || lp=$PWD/build_ab/$v
    echo "$v $(LD_LIBRARY_PATH=$lp timeout -k 10 120 shim/build/frame_bench $O/frames.u8 1241 376 8 300 20 2000 386.1448 718.856 | tail -1)" || exit 1
  done
done
for v in base $V; do
  lp=""; [ $v = base ] || lp=$PWD/build_ab/$v
  LD_LIBRARY_PATH=$lp timeout -k 10 180 rocprofv3 --kernel-trace -d $O/tr_$v -o sf -- shim/build/frame_bench $O/frames.u8 1241 376 8 100 20 2000 386.1448 718.856 > /dev/null 2>&1 || exit 1
  echo "$v trace $(python tools/single_frame_prof.py parse $O/tr_$v | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["span_us_median"],1), d["per_kernel_us_median"])')"
done
rm -f $O/frames.u8
