#!/bin/bash
# Round-5 session 16: host enqueue time vs GPU time, split vs one-graph epochs
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
OUT=gpurun_out/r5_s16_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s16.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"], "host", d["host_enqueue_ms_per_step"], d["host_launch_us_per_epoch"])')" >> $OUT; }
L="--steps 210 --warmup 21"
b long_split "$L"
b long_kadam "$L" DLAP_TAIL_ADAM=0
b long_onegraph_tailadam "$L" DLAP_SPLIT_GRAPHS=0
cat $OUT
