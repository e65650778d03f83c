#!/bin/bash
# Kernel trace of the driver-argument bench (20 timed epochs after 5 warmup) -> whole-run timeline.
set -o pipefail
TAG=${1:-ps}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 6; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_prof.log
python tools/run_timeline.py gpurun_out/${TAG}_prof --adams 21 > gpurun_out/${TAG}_runtl.txt 2>&1
python tools/timeline.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_timeline.txt 2>&1
python tools/kernel_stats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_stats.txt 2>&1
tail -3 gpurun_out/${TAG}_runtl.txt
cat gpurun_out/${TAG}_timeline.txt
rm -rf gpurun_out/${TAG}_prof
