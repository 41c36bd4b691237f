#!/bin/bash
# Round-6 call F: does config 5's LocalMapping stream share a hardware queue with the extraction
# streams?  The headline + config-5 legs at GPU_MAX_HW_QUEUES 4 (the box default) and 8, and
# config 5 with fewer extraction streams in flight.
O=gpurun_out/r6f
mkdir -p $O
A="--steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 --pipeline-steps 4 --kf-every 128"
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py $A > $O/q$q.json 2> $O/q$q.err || exit 1
  echo "q$q $(tail -1 $O/q$q.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config5"]; print(round(d["value"]), c["sequence_s"], c["extract_alone_s"], c["localba_alone_s"], c["overlap_gain"])')"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py $A --inflight $i > $O/i$i.json 2> $O/i$i.err || exit 1
  echo "inflight$i $(tail -1 $O/i$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config5"]; print(round(d["value"]), c["sequence_s"], c["extract_alone_s"], c["localba_alone_s"], c["overlap_gain"])')"
done
echo done
