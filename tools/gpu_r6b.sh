#!/bin/bash
# Round-6 measurement call B: extraction/stereo/LocalBA/pipeline GPU tests on the current library,
# LocalBA fold A/B (ba_time), LocalBA kernel stats, config-5 sequence (LocalMapping at high priority,
# two keyframe cadences).
O=gpurun_out/r6b
mkdir -p $O
R=$PWD
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_localba.py tests/test_pipeline.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for v in base nofold bdonly pponly; do
    if [ "$v" = base ]; then lib=""; else lib=$R/build_ab/$v/liborbx.so; fi
    ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4), d['iterations'], d['trials'])")"
  done
done
bash tools/ba_prof.sh 10 > $O/ba_prof.txt 2>&1 || { echo "ba_prof failed"; exit 1; }
for k in 128 256; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --ba-calls 0 --c3-steps 0 --c1-batch 0 \
    --single-frames 0 --track-steps 0 --pipeline-steps 4 --kf-every $k > $O/c5_k$k.json 2> $O/c5_k$k.err || exit 1
done
echo done
