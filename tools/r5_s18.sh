#!/bin/bash
# Round-5 session 18: unrolled split epoch graphs -- tests, A/B benches
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_invariance_gpu.py > gpurun_out/r5_s18_t1.log 2>&1 || { tail -40 gpurun_out/r5_s18_t1.log; exit 1; }
tail -2 gpurun_out/r5_s18_t1.log
OUT=gpurun_out/r5_s18_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s18.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"], "host", d["host_enqueue_ms_per_step"], d["host_launch_us_per_epoch"])')" >> $OUT; }
L="--steps 210 --warmup 21"
b long_u4 "$L"
b long_u1 "$L" DLAP_UNROLL=1
b long_u8 "$L" DLAP_UNROLL=8
b long_u16 "$L" DLAP_UNROLL=16
b short_u4 "--steps 20 --warmup 5"
b short_u1 "--steps 20 --warmup 5" DLAP_UNROLL=1
b long_u4b "$L"
b g2_u4 "--steps 60 --warmup 10 --models-per-gpu 2"
cat $OUT
