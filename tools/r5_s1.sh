#!/bin/bash
# Round-5 session 1: eval recurrences inside the fused training forward -- GPU tests, bench, knock-outs
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_invariance_gpu.py tests/test_engine_gpu.py tests/test_parity_gpu.py > gpurun_out/r5_s1_tests.log 2>&1 || { tail -30 gpurun_out/r5_s1_tests.log; exit 1; }
tail -3 gpurun_out/r5_s1_tests.log
OUT=gpurun_out/r5_s1_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s1.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT; }
b short_new "--steps 20 --warmup 5" DLAP_EVAL_IN_FWD=1
b short_old "--steps 20 --warmup 5" DLAP_EVAL_IN_FWD=0
b long_new "--steps 210 --warmup 21" DLAP_EVAL_IN_FWD=1
b long_old "--steps 210 --warmup 21" DLAP_EVAL_IN_FWD=0
b long_new_tail "--steps 210 --warmup 21" DLAP_EVAL_IN_FWD=1 DLAP_SKIP=1
b long_new_eval "--steps 210 --warmup 21" DLAP_EVAL_IN_FWD=1 DLAP_SKIP=2
b long_new_evtail "--steps 210 --warmup 21" DLAP_EVAL_IN_FWD=1 DLAP_SKIP=3
b short_new2 "--steps 20 --warmup 5" DLAP_EVAL_IN_FWD=1
cat $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s1_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r5_s1_prof.log 2>&1 || echo "rocprof failed"
ls -R gpurun_out/r5_s1_prof | head
