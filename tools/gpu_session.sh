#!/bin/bash
# One GPU session (gpurun): the GPU test suite, the default bench lines (driver-argument short run,
# 210-step steady state, two models per GPU) and an epoch timeline of the steady state.
# Usage: gpurun --timeout 1200 -- bash tools/gpu_session.sh <tag> [quick]
#   quick: skip the full test suite (invariance tests only)
set -o pipefail
tag=${1:-session}
mkdir -p gpurun_out
T="timeout -k 10"
if [ "$2" = "quick" ]; then
  $T 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_invariance_gpu.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
else
  $T 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
fi
tail -2 gpurun_out/${tag}_tests.log
OUT=gpurun_out/${tag}_bench.log; : > $OUT
b() { local name=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/${tag}_bench.err | tail -1) || { echo "[$name] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$name] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"], "host", d["host_enqueue_ms_per_step"])')" >> $OUT; }
b short "--steps 20 --warmup 5"
b long "--steps 210 --warmup 21"
b g2 "--steps 60 --warmup 10 --models-per-gpu 2"
cat $OUT
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/${tag}_prof --adams 3 --marker k_lstm_tail > gpurun_out/${tag}_timeline.txt || true
