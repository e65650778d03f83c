#!/bin/bash
# Per-kernel averages (rocprofv3 kernel trace) of one bench configuration.
# Usage: bash tools/r4_kstats.sh <tag> "<env>" <bench args...>
set -o pipefail
TAG=$1; ENVS=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py "$@" > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 6; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_prof.log | tr '\n' ' '; echo
python tools/kernel_stats.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_kstats.txt 2>&1
head -16 gpurun_out/${TAG}_kstats.txt
rm -rf gpurun_out/${TAG}_prof
