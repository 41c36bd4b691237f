#!/bin/bash
# Round-6 measurement call C: LocalBA A/B (errors_ctl one launch vs two, the fold variants) with
# per-variant HBM traffic passes; config-5 with a bounded tracking depth; extraction stage timers
# (three runs), per-kernel HBM traffic, SQ counters of k_fast (base and vslide).
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r6c
mkdir -p $O
R=$PWD
for rep in 1 2 3; do
  for v in base split nofold bdonly; do
    lib=""; opts=""
    case $v in split) opts="split_ctl=1";; nofold|bdonly) lib=$R/build_ab/$v/liborbx.so;; esac
    ORBX_LIB_OVERRIDE=$lib ORBX_TOOL_BA_OPTS=$opts timeout -k 10 120 python tools/ba_time.py 40 > $O/ba_${v}_$rep.json || exit 1
    echo "$v $(python3 -c "import json; d=json.load(open('$O/ba_${v}_$rep.json')); print(round(d['ms_per_call'],4), round(d['median_ms'],4), d['iterations'], d['trials'])")"
  done
done
for v in base nofold bdonly pponly; do
  lib=""; [ $v = base ] || lib=$R/build_ab/$v/liborbx.so
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/bat_$v/fetch -o run --output-format csv -- python3 tools/ba_time.py 10 > $O/bat_${v}_f.log 2>&1 || exit 1
  ORBX_LIB_OVERRIDE=$lib timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/bat_$v/write -o run --output-format csv -- python3 tools/ba_time.py 10 > $O/bat_${v}_w.log 2>&1 || exit 1
done
echo "ba traffic ok"
for d in 2 1; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --ba-calls 0 --c3-steps 0 --c1-batch 0 \
    --single-frames 0 --track-steps 0 --pipeline-steps 4 --kf-every 128 --c5-depth $d > $O/c5_d$d.json 2> $O/c5_d$d.err || exit 1
done
echo "c5 ok"
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > $O/stages_$rep.json 2>&1 || exit 1
  echo "base $(tail -1 $O/stages_$rep.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["stage_ms_per_step"])')"
done
OUT=$O/tn bash tools/traffic_now.sh > $O/tn.log 2>&1 || exit 1
OUT=$O/pmc_base bash tools/pmc_kernel.sh > $O/pmc_base.log 2>&1 || exit 1
ORBX_LIB_OVERRIDE=$R/build_ab/vslide/liborbx.so OUT=$O/pmc_vslide bash tools/pmc_kernel.sh > $O/pmc_vslide.log 2>&1 || exit 1
echo done
