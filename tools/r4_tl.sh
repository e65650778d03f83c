#!/bin/bash
# Steady-state one-epoch kernel timeline of the bench (kernel trace only).
set -o pipefail
TAG=${1:-tl}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 6; }
python tools/timeline.py gpurun_out/${TAG}_prof --back 3 > gpurun_out/${TAG}_timeline.txt 2>&1
cat gpurun_out/${TAG}_timeline.txt | head -70
rm -rf gpurun_out/${TAG}_prof
