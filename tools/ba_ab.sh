#!/bin/bash
# LocalBA A/B of environment knobs (GPU box): tools/ba_ab.sh "VAR=a VAR2=b" "VAR=c" ...
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/ba_time.py 30 || exit $?
done
