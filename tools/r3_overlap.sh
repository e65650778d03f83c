#!/bin/bash
# Fused LSTM + tower forward A/B: in-kernel timing and the long bench per variant.
# Usage: bash tools/r3_overlap.sh <tag>
set -o pipefail
TAG=${1:-ov}
mkdir -p gpurun_out
for V in "DLAP_RNN_OVERLAP=0" "DLAP_RNN_OVERLAP=1 DLAP_PROG_MODE=0" "DLAP_RNN_OVERLAP=1 DLAP_PROG_MODE=1"; do
  echo "== $V"
  env $V timeout -k 10 120 python -u tools/lstm_timing.py > gpurun_out/${TAG}_lt.log 2>&1 || { tail -20 gpurun_out/${TAG}_lt.log; exit 4; }
  grep -v amdgpu.ids gpurun_out/${TAG}_lt.log
  env $V timeout -k 10 200 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/${TAG}_long.log 2>&1 || { tail -20 gpurun_out/${TAG}_long.log; exit 5; }
  grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_long.log
done
