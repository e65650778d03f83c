#!/bin/bash
# Round-5 knock-out timing: steady-state epoch time with pieces of the epoch graph removed
# (wrong results, timing only) -- which parts of the epoch bound the wall time.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r5_knock.log
: > $OUT
run() {
  local tag=$1; shift
  local line
  line=$(timeout -k 10 120 env "$@" python3 bench.py --steps 210 --warmup 21 --no-ensemble9 2>>gpurun_out/r5_knock.err | tail -1) || { echo "[$tag] FAILED rc=$?" >> $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT
}
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r5_short0.log 2>&1 || exit 1
run base DLAP_SKIP=0
run tail DLAP_SKIP=1
run eval DLAP_SKIP=2
run bwd DLAP_SKIP=4
run adam DLAP_SKIP=8
run evalloss DLAP_SKIP=16
run dropmask DLAP_SKIP=32
run epochend DLAP_SKIP=64
run trainloss DLAP_SKIP=128
run eval+tail DLAP_SKIP=3
run eval+adam DLAP_SKIP=10
run base2 DLAP_SKIP=0
cat $OUT
