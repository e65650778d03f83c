#!/bin/bash
# GPU suite, then LSTM in-kernel timing, the PMC passes and the 9-model bench.
# Usage: bash tools/r3_perf.sh <tag>
set -o pipefail
TAG=${1:-pf}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/${TAG}_tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 120 python -u tools/lstm_timing.py > gpurun_out/${TAG}_lstm.log 2>&1 || { tail -20 gpurun_out/${TAG}_lstm.log; exit 4; }
cat gpurun_out/${TAG}_lstm.log
timeout -k 10 200 python -u bench.py --models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${TAG}_g9.log 2>&1 || { tail -20 gpurun_out/${TAG}_g9.log; exit 5; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_g9.log
bash tools/pmc_final.sh ${TAG} > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 6; }
python tools/pmc_summary.py gpurun_out/${TAG}_pmc1 gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_pmc3 > gpurun_out/${TAG}_pmc_summary.txt 2>&1
rm -rf gpurun_out/${TAG}_pmc1 gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_pmc3
grep -A12 "k_mlp_bwd_sdf\|== .*k_mlp_fwd" gpurun_out/${TAG}_pmc_summary.txt | head -60
