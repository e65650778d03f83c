#!/bin/bash
# Final-tree evidence: kernel stats of the headline bench, 9-model batching, scaled panel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o prof -- python3 bench.py --no-ensemble9 > gpurun_out/fin_bench_prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --models-per-gpu 9 --no-ensemble9 > gpurun_out/fin_bench_g9.log 2>&1 && \
timeout -k 10 500 python -u bench.py --config scaled --steps 42 --warmup 6 > gpurun_out/fin_bench_scaled.log 2>&1
