# Gram build grid A/B (DLAP_GRAM_WG) on the driver-argument run, with kernel trace durations
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6s}
for wg in 256 512 1024 2048; do
  DLAP_GRAM_WG=$wg $T 300 python bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  echo "wg=$wg $(tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' ')"
  DLAP_GRAM_WG=$wg $T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_p$wg -o run -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/${tag}_p$wg.log 2>&1 || { tail -5 gpurun_out/${tag}_p$wg.log; exit 1; }
  python3 tools/kernel_stats.py gpurun_out/${tag}_p$wg > gpurun_out/${tag}_ks$wg.txt 2>&1 || true
  rm -rf gpurun_out/${tag}_p$wg
  grep "k_gram" gpurun_out/${tag}_ks$wg.txt | cut -c1-110
done
