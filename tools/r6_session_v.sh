# loss-pass issue priority A/B
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6v}
for p in 0 1 0 1; do
for a in "--steps 210 --warmup 21" "--steps 20 --warmup 5"; do
  DLAP_LOSS_PRIO=$p $T 300 python bench.py $a --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  echo "prio=$p $a $(tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' ')"
done
done
