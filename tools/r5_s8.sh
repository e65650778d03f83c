#!/bin/bash
# Round-5 session 8: kernel trace of the default tree (epoch timeline + kernel table)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_s8_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/r5_s8_prof.log 2>&1 || { tail -20 gpurun_out/r5_s8_prof.log; exit 1; }
tail -1 gpurun_out/r5_s8_prof.log
python3 tools/run_timeline.py gpurun_out/r5_s8_prof --adams 3 > gpurun_out/r5_s8_timeline.txt
cat gpurun_out/r5_s8_timeline.txt | head -60
