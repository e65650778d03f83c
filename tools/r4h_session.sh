#!/bin/bash
# Round-4 session H: Gram build with double-buffered loads: numerics, then kernel time + bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gram_gpu.py > gpurun_out/r4h_gram.log 2>&1 \
  || { echo "gram tests FAILED"; tail -30 gpurun_out/r4h_gram.log; exit 3; }
grep -E "PASSED|FAILED" gpurun_out/r4h_gram.log
bash tools/r4_ab.sh r4h "s_def||--steps 20 --warmup 5 --no-ensemble9" "l_def||--steps 210 --warmup 21 --no-ensemble9" && \
bash tools/r4_kstats.sh r4hk1 "" --steps 20 --warmup 5 --no-ensemble9 && grep -E "gram" gpurun_out/r4hk1_kstats.txt
