#!/bin/bash
# Fused Adam re-pack: its equivalence test, the engine-vs-torch tests, short and default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_invariance_gpu.py tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r4_fp_tests.log 2>&1 \
  || { echo "tests FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r4_fp_tests.log | tail -20; tail -5 gpurun_out/r4_fp_tests.log; exit 3; }
tail -2 gpurun_out/r4_fp_tests.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r4_fp_short$i.log 2>&1 || { tail -20 gpurun_out/r4_fp_short$i.log; exit 5; }
  tail -1 gpurun_out/r4_fp_short$i.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py > gpurun_out/r4_fp_default.log 2>&1 || { tail -20 gpurun_out/r4_fp_default.log; exit 5; }
tail -1 gpurun_out/r4_fp_default.log
bash tools/r3_prof_short.sh r4fp > gpurun_out/r4fp_prof_summary.txt 2>&1 || exit 7
