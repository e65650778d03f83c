#!/bin/bash
# GPU test suite (stops at the first failure) + the driver-argument bench + the long bench.
# Usage: bash tools/r3_check.sh <tag> [pytest selection...]
set -o pipefail
TAG=${1:-chk}; shift
SEL=${@:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 3; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_short.log 2>&1 || { tail -20 gpurun_out/${TAG}_short.log; exit 4; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]\|"wall_s": [0-9.]*' gpurun_out/${TAG}_short.log
timeout -k 10 200 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/${TAG}_long.log 2>&1 || { tail -20 gpurun_out/${TAG}_long.log; exit 5; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_long.log
