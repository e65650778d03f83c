#!/bin/bash
# Round-4 session N: 32-bit tile-load offsets in the tower kernels: invariance + engine tests, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_invariance_gpu.py \
  tests/test_engine_gpu.py tests/test_engine_fp32_gpu.py tests/test_gram_gpu.py > gpurun_out/r4n_tests.log 2>&1 \
  || { echo "tests FAILED"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r4n_tests.log | tail -30; exit 3; }
grep -cE "PASSED" gpurun_out/r4n_tests.log; grep -E "FAILED" gpurun_out/r4n_tests.log | head
bash tools/r4_ab.sh r4n "s_def||--steps 20 --warmup 5 --no-ensemble9" "l_def||--steps 210 --warmup 21 --no-ensemble9" \
  "g9_def||--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" "sc_def||--config scaled --steps 20 --warmup 5 --no-ensemble9"
