#!/bin/bash
# Full GPU test suite (one process) + smoke + a driver-argument bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_full_gpu_tests.log 2>&1 \
  || { echo "GPU suite FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r4_full_gpu_tests.log | tail -20; tail -5 gpurun_out/r4_full_gpu_tests.log; exit 3; }
tail -3 gpurun_out/r4_full_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 4; }
tail -1 gpurun_out/r4_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4_bench_default.log 2>&1 || { tail -20 gpurun_out/r4_bench_default.log; exit 5; }
tail -1 gpurun_out/r4_bench_default.log
