#!/bin/bash
# Early vs late dropout-mask generation in the pipelined epoch: invariance / dropout tests, then
# driver-argument and steady bench lines with DLAP_EARLY_DROPMASK=1 (default) and =0.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_invariance_gpu.py tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4_dm_tests.log 2>&1 \
  || { echo "tests FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r4_dm_tests.log | tail -20; exit 3; }
tail -1 gpurun_out/r4_dm_tests.log
for v in 1 0 1 0; do
  DLAP_EARLY_DROPMASK=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r4_dm_s$v.log 2>&1 || { tail -20 gpurun_out/r4_dm_s$v.log; exit 5; }
  echo "early=$v short $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_dm_s$v.log)"
  DLAP_EARLY_DROPMASK=$v timeout -k 10 200 python -u bench.py --no-ensemble9 > gpurun_out/r4_dm_l$v.log 2>&1 || { tail -20 gpurun_out/r4_dm_l$v.log; exit 5; }
  echo "early=$v long $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4_dm_l$v.log)"
done
bash tools/r3_prof_short.sh r4dm > gpurun_out/r4dm_prof_summary.txt 2>&1 || exit 7
