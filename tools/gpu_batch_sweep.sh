#!/bin/bash
# Headline bench at several frames-per-step / batches-in-flight settings (extract + match only)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/batch_sweep
mkdir -p $O
for rep in 1 2; do
  for cfg in "256 4" "512 4" "512 2" "1024 2" "128 8"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --batch $1 --inflight $2 --steps 10 --warmup 2 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 > $O/b$1_i$2_$rep.log 2>&1 || { echo "B=$1 I=$2 failed"; tail -5 $O/b$1_i$2_$rep.log; exit 1; }
    echo "B=$1 I=$2 $(tail -1 $O/b$1_i$2_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["ms_per_step"])')"
  done
done
