#!/bin/bash
# Client-side wait for a free GPU slot: re-submits the SAME command only while gpurun reports that
# nothing ran (no slot / box prepared badly, "nothing was charged" or charged=0.0s); any call that
# actually ran (pass or fail) ends the loop.  Usage: tools/gpu_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TMO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  if grep -q "charged=0.0s\|nothing was charged\|backing off" "$LOG" && ! grep -q "status=ok\|status=fail" "$LOG"; then
    sleep 75
    continue
  fi
  break
done
