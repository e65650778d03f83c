#!/bin/bash
# Kernel + HIP API trace of the driver-argument bench: where the GPU idles at graph boundaries.
set -o pipefail
TAG=${1:-ht}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 6; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_prof.log
python tools/host_gaps.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_hostgaps.txt 2>&1
python tools/run_timeline.py gpurun_out/${TAG}_prof --adams 21 > gpurun_out/${TAG}_runtl.txt 2>&1
tail -22 gpurun_out/${TAG}_hostgaps.txt
tail -1 gpurun_out/${TAG}_runtl.txt
rm -rf gpurun_out/${TAG}_prof
