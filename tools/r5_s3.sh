#!/bin/bash
# Round-5 session 3: fused tail with W_ih helper blocks -- bitwise tests, in-kernel timing, benches
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_invariance_gpu.py tests/test_engine_gpu.py -k "fused_backward_tail or eval_recurrences or poisons or pipelined or deterministic or replay or batching" > gpurun_out/r5_s3_t1.log 2>&1 || { tail -40 gpurun_out/r5_s3_t1.log; exit 1; }
tail -3 gpurun_out/r5_s3_t1.log
$T 200 python3 tools/lstm_timing.py > gpurun_out/r5_s3_lstm_timing.txt 2>&1 || { cat gpurun_out/r5_s3_lstm_timing.txt; exit 1; }
cat gpurun_out/r5_s3_lstm_timing.txt
OUT=gpurun_out/r5_s3_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s3.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT; }
b short_new "--steps 20 --warmup 5"
b long_new "--steps 210 --warmup 21"
b long_notail "--steps 210 --warmup 21" DLAP_FUSED_TAIL=0
b long_new_noeval "--steps 210 --warmup 21" DLAP_SKIP=2
b short_new2 "--steps 20 --warmup 5"
cat $OUT
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s3_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r5_s3_prof.log 2>&1 || echo "rocprof failed"
