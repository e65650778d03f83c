#!/bin/bash
# Round-5 session 13: tail Adam with running counts and pre-read step counters
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_invariance_gpu.py > gpurun_out/r5_s13_t1.log 2>&1 || { tail -40 gpurun_out/r5_s13_t1.log; exit 1; }
tail -2 gpurun_out/r5_s13_t1.log
$T 200 python3 tools/lstm_timing.py > gpurun_out/r5_s13_timing.txt 2>&1 || { tail gpurun_out/r5_s13_timing.txt; exit 1; }
grep -A12 "pipeline=True" gpurun_out/r5_s13_timing.txt
OUT=gpurun_out/r5_s13_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s13.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT; }
L="--steps 210 --warmup 21"
b long_new "$L"
b long_kadam "$L" DLAP_TAIL_ADAM=0
b long_new2 "$L"
b long_kadam2 "$L" DLAP_TAIL_ADAM=0
cat $OUT
