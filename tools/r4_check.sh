#!/bin/bash
# Round-4 check on the GPU box: the invariance / fused-safety tests, the whole GPU suite, the
# driver-argument bench (x2), the steady-state bench and 9 batched models.
# Usage (GPU box): bash tools/r4_check.sh <tag>   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-r4}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_invariance_gpu.py tests/test_panel_gpu.py -x -s -v -rfE --timeout 200 --timeout-method thread > gpurun_out/${TAG}_inv.log 2>&1 || { tail -40 gpurun_out/${TAG}_inv.log; exit 3; }
tail -1 gpurun_out/${TAG}_inv.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfE --timeout 200 --timeout-method thread --deselect tests/test_invariance_gpu.py --deselect tests/test_panel_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 4; }
tail -1 gpurun_out/${TAG}_tests.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_short$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_short$r.log; exit 5; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]\|"wall_s": [0-9.]*\|"test_sharpe": [0-9.-]*' gpurun_out/${TAG}_short$r.log | tr '\n' ' '; echo
done
timeout -k 10 200 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/${TAG}_long.log 2>&1 || { tail -20 gpurun_out/${TAG}_long.log; exit 6; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_long.log | tr '\n' ' '; echo
timeout -k 10 200 python -u bench.py --models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${TAG}_g9.log 2>&1 || { tail -20 gpurun_out/${TAG}_g9.log; exit 7; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/${TAG}_g9.log | tr '\n' ' '; echo
