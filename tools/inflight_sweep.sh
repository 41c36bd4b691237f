#!/bin/bash
# headline step vs batches in flight (streams): 4 (default), 6, 8, 3
mkdir -p gpurun_out
for n in 4 6 8 3 4; do
  timeout -k 10 300 python bench.py --inflight $n --steps 40 --warmup 8 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > gpurun_out/inflight_$n.json 2>&1 || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/inflight_$n.json').read().strip().splitlines()[-1]);print($n, d['value'], d['ms_per_step'], d['median_ms_per_step'])" >> gpurun_out/inflight.txt
done
