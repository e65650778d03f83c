#!/bin/bash
# Bench at the driver's arguments and at the long default, plus a kernel trace of the short run.
# Usage: bash tools/r3_baseline.sh <tag> [extra env assignments]
set -o pipefail
TAG=${1:-base}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
env "$@" timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_short.log 2>&1 || { tail -20 gpurun_out/${TAG}_short.log; exit 4; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]\|"wall_s": [0-9.]*' gpurun_out/${TAG}_short.log
env "$@" timeout -k 10 200 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/${TAG}_long.log 2>&1 || { tail -20 gpurun_out/${TAG}_long.log; exit 5; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_long.log
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 105 --warmup 12 --no-ensemble9 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 6; }
python tools/kernel_stats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_stats.txt 2>&1
python tools/timeline.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_timeline.txt 2>&1
cat gpurun_out/${TAG}_timeline.txt
rm -rf gpurun_out/${TAG}_prof
