#!/bin/bash
# Benches only (after the tests passed): driver-argument bench x2, steady state, 9 batched
# models, then the kernel + HIP API trace of the driver-argument run.
set -o pipefail
TAG=${1:-r4}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_short$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_short$r.log; exit 5; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]\|"wall_s": [0-9.]*\|"test_sharpe": [0-9.-]*\|"panel_compaction": [0-9.]*\|"train_total": [0-9.]*\|"epochs": [0-9.]*\|"gram_plan": \[[^]]*\]\]' gpurun_out/${TAG}_short$r.log | tr '\n' ' '; echo
done
timeout -k 10 200 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/${TAG}_long.log 2>&1 || { tail -20 gpurun_out/${TAG}_long.log; exit 6; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_long.log | tr '\n' ' '; echo
timeout -k 10 200 python -u bench.py --models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${TAG}_g9.log 2>&1 || { tail -20 gpurun_out/${TAG}_g9.log; exit 7; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/${TAG}_g9.log | tr '\n' ' '; echo
bash tools/r4_hiptrace.sh ${TAG}h || exit 8
