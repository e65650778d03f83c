#!/bin/bash
# One GPU iteration: GPU tests, the headline bench, and a kernel trace summarised into a kernel
# table + one-epoch timeline (gpurun_out/<tag>_stats.txt, <tag>_timeline.txt).
# Usage: bash tools/gpu_perf.sh <tag> [extra env assignments for the bench/profile]
set -o pipefail
TAG=${1:-perf}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 3; }
tail -2 gpurun_out/${TAG}_tests.log
env "$@" timeout -k 10 200 python -u bench.py --steps 105 --warmup 12 --no-ensemble9 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 4; }
grep -o '"value": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_bench.log
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 105 --warmup 12 --no-ensemble9 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 5; }
python tools/kernel_stats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_stats.txt 2>&1
python tools/timeline.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_timeline.txt 2>&1
cat gpurun_out/${TAG}_timeline.txt
rm -rf gpurun_out/${TAG}_prof
