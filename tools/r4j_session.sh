#!/bin/bash
# Round-4 session J: dense-state LSTM BPTT + unrolled pre-pass: numerics, in-kernel timing, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lstm_bptt_gpu.py \
  tests/test_engine_gpu.py tests/test_engine_fp32_gpu.py tests/test_module_autograd_gpu.py > gpurun_out/r4j_tests.log 2>&1 \
  || { echo "tests FAILED"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r4j_tests.log | tail -30; exit 3; }
grep -cE "PASSED" gpurun_out/r4j_tests.log; grep -E "FAILED|SKIPPED" gpurun_out/r4j_tests.log | head
timeout -k 10 200 python -u tools/lstm_timing.py > gpurun_out/r4j_lstm_timing.txt 2>&1 || { tail -20 gpurun_out/r4j_lstm_timing.txt; exit 4; }
grep -E "pipeline|k_lstm_bwd|recur" gpurun_out/r4j_lstm_timing.txt
DLAP_LSTM_SCAN=0 timeout -k 10 200 python -u tools/lstm_timing.py > gpurun_out/r4j_lstm_timing_old.txt 2>&1 || exit 5
grep -E "pipeline|k_lstm_bwd" gpurun_out/r4j_lstm_timing_old.txt
bash tools/r4_ab.sh r4j "s_def||--steps 20 --warmup 5 --no-ensemble9" "l_def||--steps 210 --warmup 21 --no-ensemble9" \
  "s_old|DLAP_LSTM_SCAN=0|--steps 20 --warmup 5 --no-ensemble9" "g9_def||--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9"
