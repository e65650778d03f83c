#!/bin/bash
# Round-5 session 2: eval recurrences in the fused forward + fused backward tail: bitwise tests,
# A/B benches, kernel trace, remaining GPU tests
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_invariance_gpu.py -k "fused_backward_tail or eval_recurrences" > gpurun_out/r5_s2_t1.log 2>&1 || { tail -40 gpurun_out/r5_s2_t1.log; exit 1; }
tail -3 gpurun_out/r5_s2_t1.log
OUT=gpurun_out/r5_s2_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s2.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT; }
b short_new "--steps 20 --warmup 5"
b short_evonly "--steps 20 --warmup 5" DLAP_FUSED_TAIL=0
b short_old "--steps 20 --warmup 5" DLAP_EVAL_IN_FWD=0 DLAP_FUSED_TAIL=0
b long_new "--steps 210 --warmup 21"
b long_evonly "--steps 210 --warmup 21" DLAP_FUSED_TAIL=0
b long_tailonly "--steps 210 --warmup 21" DLAP_EVAL_IN_FWD=0
b long_old "--steps 210 --warmup 21" DLAP_EVAL_IN_FWD=0 DLAP_FUSED_TAIL=0
b long_new_noeval "--steps 210 --warmup 21" DLAP_SKIP=2
b long_new_notail "--steps 210 --warmup 21" DLAP_SKIP=1
b short_new2 "--steps 20 --warmup 5"
cat $OUT
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s2_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r5_s2_prof.log 2>&1 || echo "rocprof failed"
$T 1100 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_invariance_gpu.py tests/test_parity_gpu.py tests/test_lstm_bptt_gpu.py tests/test_engine_fp32_gpu.py > gpurun_out/r5_s2_tests.log 2>&1
tail -8 gpurun_out/r5_s2_tests.log
