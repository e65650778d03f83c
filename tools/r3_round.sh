#!/bin/bash
# Full GPU suite (no -x: every failure listed), optional debug script, the driver-argument bench
# and the long bench. Usage: bash tools/r3_round.sh <tag> [debug-script]
set -o pipefail
TAG=${1:-rd}
DBG=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$DBG" ]; then
  timeout -k 10 240 python -u $DBG > gpurun_out/${TAG}_dbg.log 2>&1
  rc=$?; tail -30 gpurun_out/${TAG}_dbg.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 2; fi
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/${TAG}_tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_short.log 2>&1 || { tail -20 gpurun_out/${TAG}_short.log; exit 4; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]\|"wall_s": [0-9.]*' gpurun_out/${TAG}_short.log
timeout -k 10 200 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/${TAG}_long.log 2>&1 || { tail -20 gpurun_out/${TAG}_long.log; exit 5; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_long.log
