#!/bin/bash
# Round-6 call E: extraction/stereo/LocalBA/pipeline GPU tests on the current library (k_fast cell
# loop unrolled, compact candidate slots, two-launch LM verdict), stage timers A/B against the full
# per-cell candidate layout (three alternating rounds), LocalBA call time (default vs fused_ctl),
# SQ counters of the current k_fast and of the vslide variant.
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r6e
mkdir -p $O
R=$PWD
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_localba.py tests/test_pipeline.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in base oldcand; do
    lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > $O/stages_${v}_$rep.json 2>&1 || exit 1
    echo "$v $(tail -1 $O/stages_${v}_$rep.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["stage_ms_per_step"])')"
  done
done
for rep in 1 2 3; do
  for v in base fused; do
    opts=""; [ $v = fused ] && opts="fused_ctl=1"
    ORBX_TOOL_BA_OPTS=$opts timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4), d['iterations'], d['trials'])")"
  done
done
OUT=$O/pmc_base bash tools/pmc_kernel.sh > $O/pmc_base.log 2>&1 || exit 1
ORBX_LIB_OVERRIDE=$R/build_ab/vslide/liborbx.so OUT=$O/pmc_vslide bash tools/pmc_kernel.sh > $O/pmc_vslide.log 2>&1 || exit 1
echo done
