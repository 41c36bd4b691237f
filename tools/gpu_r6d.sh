#!/bin/bash
# Round-6 measurement call D: GPU tests on the current library; errors_ctl A/B (release per block +
# acquire fence in the last block [base], acq_rel in every block, the two-launch form); compact FAST
# candidate slots A/B against the full per-cell layout (stage timers, alternating, three rounds);
# SQ counters of the vslide k_fast variant.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r6d
mkdir -p $O
R=$PWD
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_localba.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in base acqrel split nofold; do
    lib=""; opts=""
    case $v in split) opts="split_ctl=1";; acqrel|nofold) lib=$R/build_ab/$v/liborbx.so;; esac
    ORBX_LIB_OVERRIDE=$lib ORBX_TOOL_BA_OPTS=$opts timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4), d['iterations'], d['trials'])")"
  done
done
for rep in 1 2 3; do
  for v in base oldcand; do
    lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > $O/stages_${v}_$rep.json 2>&1 || exit 1
    echo "$v $(tail -1 $O/stages_${v}_$rep.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["stage_ms_per_step"])')"
  done
done
ORBX_LIB_OVERRIDE=$R/build_ab/vslide/liborbx.so OUT=$O/pmc_vslide bash tools/pmc_kernel.sh > $O/pmc_vslide.log 2>&1 || exit 1
echo done
