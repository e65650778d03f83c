#!/bin/bash
# End-of-session evidence: GPU suite, smoke, driver-argument bench (x2), long bench, 9 batched
# models, scaled panel, kernel-trace timeline + stats of the driver-argument run, PMC passes.
# Usage (GPU box): bash tools/r3_final.sh <tag>   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-fin}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rfE --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 3; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 4; }
tail -1 gpurun_out/${TAG}_smoke.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_short$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_short$r.log; exit 5; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"wall_s": [0-9.]*' gpurun_out/${TAG}_short$r.log | tr '\n' ' '; echo
done
timeout -k 10 200 python -u bench.py --steps 210 --warmup 21 --no-ensemble9 > gpurun_out/${TAG}_long.log 2>&1 || { tail -20 gpurun_out/${TAG}_long.log; exit 6; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_long.log | tr '\n' ' '; echo
timeout -k 10 200 python -u bench.py --models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${TAG}_g9.log 2>&1 || { tail -20 gpurun_out/${TAG}_g9.log; exit 7; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/${TAG}_g9.log | tr '\n' ' '; echo
timeout -k 10 400 python -u bench.py --config scaled --steps 21 --warmup 6 > gpurun_out/${TAG}_scaled.log 2>&1 || { tail -20 gpurun_out/${TAG}_scaled.log; exit 8; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' gpurun_out/${TAG}_scaled.log | tr '\n' ' '; echo
bash tools/r3_prof_short.sh ${TAG}p > gpurun_out/${TAG}p.out 2>&1 || { tail -5 gpurun_out/${TAG}p.out; exit 9; }
head -3 gpurun_out/${TAG}p.out | tr '\n' ' '; echo
bash tools/pmc_final.sh ${TAG} > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 10; }
python tools/pmc_summary.py gpurun_out/${TAG}_pmc1 gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_pmc3 > gpurun_out/${TAG}_pmc_summary.txt 2>&1
rm -rf gpurun_out/${TAG}_pmc1 gpurun_out/${TAG}_pmc2 gpurun_out/${TAG}_pmc3
grep -A4 "== void k_mlp_bwd_sdf<PrecBF16, 2, 2, 2\|== void k_mlp_fwd_rnn\|== void k_mlp_fwd<PrecBF16, 2, 1" gpurun_out/${TAG}_pmc_summary.txt | grep -E "==|VALU |MFMA " | head -12
