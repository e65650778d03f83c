#!/bin/bash
# Round-5 session 15: host/GPU interleaving of the split epoch graphs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d gpurun_out/r5_s15_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/r5_s15_prof.log 2>&1 || { tail -5 gpurun_out/r5_s15_prof.log; exit 1; }
python3 tools/host_gaps.py gpurun_out/r5_s15_prof --adams 4 --marker k_lstm_tail > gpurun_out/r5_s15_hostgaps.txt || true
head -80 gpurun_out/r5_s15_hostgaps.txt
