#!/bin/bash
# Round-4 session L: dense-state BPTT (pair links) + MFMA LSTM weight gradients.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lstm_bptt_gpu.py \
  tests/test_engine_gpu.py tests/test_engine_fp32_gpu.py tests/test_module_autograd_gpu.py tests/test_dropout_gpu.py > gpurun_out/r4l_tests.log 2>&1 \
  || { echo "tests FAILED"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r4l_tests.log | tail -30; exit 3; }
grep -cE "PASSED" gpurun_out/r4l_tests.log; grep -E "FAILED|SKIPPED" gpurun_out/r4l_tests.log | head
timeout -k 10 200 python -u tools/lstm_timing.py > gpurun_out/r4l_lstm_timing.txt 2>&1 || { tail -20 gpurun_out/r4l_lstm_timing.txt; exit 4; }
grep -E "pipeline|k_lstm_bwd|dense" gpurun_out/r4l_lstm_timing.txt
bash tools/r4_ab.sh r4l "s_def||--steps 20 --warmup 5 --no-ensemble9" "l_def||--steps 210 --warmup 21 --no-ensemble9" \
  "s_old|DLAP_LSTM_SCAN=0|--steps 20 --warmup 5 --no-ensemble9" "s_def2||--steps 20 --warmup 5 --no-ensemble9"
