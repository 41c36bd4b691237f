#!/bin/bash
# Round-6 call H: config 5 with LocalMapping and Tracking on disjoint CU sets (CU-masked streams):
# LocalBA CUs 32 / 64 / 96, contiguous and strided, against the shared GPU.
O=gpurun_out/r6h
mkdir -p $O
A="--steps 5 --warmup 2 --no-cpu-baseline --ba-calls 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 --pipeline-steps 4 --kf-every 128"
run() {
  timeout -k 10 300 python bench.py $A "$@" > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
  echo "$tag $(tail -1 $O/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config5"]; print(c["frames_per_s_sequence"], c["sequence_s"], c["extract_alone_s"], c["localba_alone_s"], c["overlap_gain"])')"
}
tag=shared run
for n in 32 64 96; do
  for lay in contiguous strided; do
    tag=cu${n}_$lay run --c5-ba-cus $n --c5-cu-layout $lay
  done
done
echo done
