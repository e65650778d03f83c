#!/bin/bash
# Gram-mode tests, then the r3 baseline bench/profile, then an A/B of the long bench with DLAP_GRAM=0.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gram_gpu.py tests/test_engine_fp32_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gram_tests.log 2>&1 || { tail -40 gpurun_out/gram_tests.log; exit 3; }
tail -3 gpurun_out/gram_tests.log
bash tools/r3_baseline.sh gram || exit $?
timeout -k 10 200 env DLAP_GRAM=0 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/nogram_long.log 2>&1 || exit 7
grep -o '"value": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/nogram_long.log
