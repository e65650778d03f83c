# scaled panel: bench A/B (8 vs 16 waves in the streamed wide forward), kernel timeline, SQ counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6y}
for w in 8 16; do
  DLAP_ZX_WAVES=$w $T 400 python bench.py --config scaled --steps 20 --warmup 5 > gpurun_out/${tag}_w$w.log 2>&1 || { tail -20 gpurun_out/${tag}_w$w.log; exit 1; }
  echo "waves=$w"; tail -1 gpurun_out/${tag}_w$w.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' '; echo
done
$T 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_sprof -o run -- python3 bench.py --config scaled --steps 10 --warmup 3 > gpurun_out/${tag}_sprof.log 2>&1 || { tail -5 gpurun_out/${tag}_sprof.log; exit 1; }
python3 tools/kernel_stats.py gpurun_out/${tag}_sprof > gpurun_out/${tag}_scaled_kernels.txt 2>&1 || true
python3 tools/run_timeline.py gpurun_out/${tag}_sprof --adams 3 --marker k_lstm_tail > gpurun_out/${tag}_scaled_timeline.txt 2>&1 || true
head -30 gpurun_out/${tag}_scaled_kernels.txt
$T 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/${tag}_spmc -o run -- python3 bench.py --config scaled --steps 6 --warmup 2 > gpurun_out/${tag}_spmc.log 2>&1 || { tail -5 gpurun_out/${tag}_spmc.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/${tag}_spmc > gpurun_out/${tag}_scaled_pmc.txt 2>&1 || true
head -40 gpurun_out/${tag}_scaled_pmc.txt
