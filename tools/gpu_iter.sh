#!/bin/bash
# round-4 iteration on the GPU box: the given test files (default: extraction, stereo, tracking), then a
# short headline bench (stage split) -> gpurun_out/iter_*.  A crash, abort or time limit ends the call.
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_tracking.py}
timeout -k 10 400 python -u -m pytest $TESTS -q -x --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/iter_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --ba-calls ${BA_CALLS:-0} --pipeline-steps 0 --c3-steps 0 --single-frames 0 --track-steps 0 ${BENCH_EXTRA:-} > gpurun_out/iter_bench.json 2> gpurun_out/iter_bench.err
brc=$?
echo "bench rc=$brc"
python3 -c "import json;d=json.loads(open('gpurun_out/iter_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['stage_ms_per_step'])" || tail -c 1500 gpurun_out/iter_bench.err
[ $brc -eq 0 ] || exit $brc
# batch-shape sweep (headline only): smaller batches keep a batch's levels inside the 256 MB MALL
for bf in ${SWEEP:-}; do
  b=${bf%x*}; f=${bf#*x}
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --batch $b --inflight $f --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --single-frames 0 --track-steps 0 --profile-steps 2 > gpurun_out/iter_sweep_$bf.json 2>/dev/null || exit $?
  echo "sweep $bf $(python3 -c "import json;d=json.loads(open('gpurun_out/iter_sweep_$bf.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
exit $rc
