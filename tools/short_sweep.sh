#!/bin/bash
# A/B of engine knobs on the driver-argument bench (--steps 20 --warmup 5), arms interleaved
# twice. Usage: gpurun -- bash tools/short_sweep.sh <tag> "NAME=V" ... ("-" = defaults)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/${tag}.log; : > $OUT
for rep in 1 2; do
  for arm in "$@"; do
    kv=$arm; [ "$arm" = "-" ] && kv="X_DEFAULT=1"
    line=$(timeout -k 10 200 env $kv python3 bench.py --steps 20 --warmup 5 --no-ensemble9 2>>gpurun_out/${tag}.err | tail -1) || { echo "[$arm] FAILED" >> $OUT; cat $OUT; exit 1; }
    echo "[$arm] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT
  done
done
cat $OUT
