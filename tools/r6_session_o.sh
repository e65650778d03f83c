# Gram plan A/B on the driver-argument run and the steady state
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6o}
for env in "DLAP_GRAM_PLAN=1" "DLAP_GRAM_PLAN=2" "DLAP_GRAM_PLAN=3" "DLAP_GRAM=0"; do
for a in "--steps 20 --warmup 5" "--steps 210 --warmup 21"; do
  env $env $T 300 python bench.py $a --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  echo "$env $a $(tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]\|"gram_plan": \[[^]]*\]\]' | tr '\n' ' ')"
done
done
