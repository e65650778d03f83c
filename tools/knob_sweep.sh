#!/bin/bash
# A/B sweep of engine knobs on the steady-state bench (one GPU). Usage:
#   gpurun -- bash tools/knob_sweep.sh <tag> "NAME=V ..." "NAME=V ..." ...   ("-" = defaults)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/${tag}.log; : > $OUT
for arm in "$@"; do
  kv=$arm; [ "$arm" = "-" ] && kv="X_DEFAULT=1"
  line=$(timeout -k 10 200 env $kv python3 bench.py --steps 210 --warmup 21 --no-ensemble9 2>>gpurun_out/${tag}.err | tail -1) || { echo "[$arm] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$arm] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT
done
cat $OUT
