#!/bin/bash
# Round-4 evidence: multi-rank rehearsal (gloo, one GPU), the BASELINE config-4 grid on one
# GPU, a cross-sectional (N-sharded) timing line and the instruction-mix / bank-conflict PMC.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/r4_rehearse.sh r4e || exit 3
timeout -k 10 400 python -u -m deeplearninginassetpricing_paperreplication_amd.parallel.sweep --synthetic 240 60 300 3000 46 178 --grid baseline > gpurun_out/r4e_sweep_baseline.log 2>&1 || { tail -20 gpurun_out/r4e_sweep_baseline.log; exit 4; }
tail -1 gpurun_out/r4e_sweep_baseline.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('n_configs','n_buckets','n_ok','wall_s','predicted_imbalance','best_point','best_valid_sharpe','best_test_sharpe','stage_s_local')})"
timeout -k 10 300 python -u -m deeplearninginassetpricing_paperreplication_amd.parallel.xsection --synthetic 240 60 300 3000 46 178 --epochs 16 4 32 --ignore_epoch 2 --print_freq 1000 > gpurun_out/r4e_xsection.log 2>&1 || { tail -20 gpurun_out/r4e_xsection.log; exit 5; }
tail -1 gpurun_out/r4e_xsection.log
bash tools/pmc_final.sh r4e > gpurun_out/r4e_pmc.log 2>&1 || { tail -20 gpurun_out/r4e_pmc.log; exit 6; }
python tools/pmc_summary.py gpurun_out/r4e_pmc1 gpurun_out/r4e_pmc2 gpurun_out/r4e_pmc3 > gpurun_out/r4e_pmc_summary.txt 2>&1
rm -rf gpurun_out/r4e_pmc1 gpurun_out/r4e_pmc2 gpurun_out/r4e_pmc3
grep -A12 "== void k_mlp_bwd_sdf<PrecBF16, 2, 2, 1, false, 1>" gpurun_out/r4e_pmc_summary.txt | head -30
