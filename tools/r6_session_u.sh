# G=2 evaluation grid A/B (steady state)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6u}
for gx in 128 192 256 384; do
  DLAP_EVAL_GX=$gx $T 300 python bench.py --steps 210 --warmup 21 --no-ensemble9 --models-per-gpu 2 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  echo "G=2 eval_gx=$gx $(tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' ')"
done
