#!/bin/bash
# extraction/stereo GPU parity tests, then a short bench (no CPU baseline, no LocalBA/side legs)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_stereo.py tests/test_golden.py tests/test_shim.py tests/test_tracking.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ext_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ext_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --ba-calls 0 ${BENCH_EXTRA} > gpurun_out/bench_ext.log 2>&1
rc=$?; echo "bench rc=$rc"
python - <<'PY'
import json
j = json.loads(open("gpurun_out/bench_ext.log").read().strip().splitlines()[-1])
print("value", j["value"], "ms/step", j["ms_per_step"], "median", j["median_ms_per_step"])
print(json.dumps(j["stage_ms_per_step"]))
PY
exit $rc
