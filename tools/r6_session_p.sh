# scaled panel on the current tree (bench + kernel stats), Gram build counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6p}
$T 400 python bench.py --config scaled --steps 20 --warmup 5 > gpurun_out/${tag}_scaled.log 2>&1 || { tail -20 gpurun_out/${tag}_scaled.log; exit 1; }
tail -1 gpurun_out/${tag}_scaled.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' '; echo
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_sprof -o run -- python3 bench.py --config scaled --steps 10 --warmup 3 > gpurun_out/${tag}_sprof.log 2>&1 || { tail -5 gpurun_out/${tag}_sprof.log; exit 1; }
python3 tools/kernel_stats.py gpurun_out/${tag}_sprof > gpurun_out/${tag}_scaled_kernels.txt 2>&1 || true
head -25 gpurun_out/${tag}_scaled_kernels.txt
$T 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS --kernel-trace -d gpurun_out/${tag}_gpmc -o run -- python3 bench.py --steps 10 --warmup 3 --no-ensemble9 > gpurun_out/${tag}_gpmc.log 2>&1 || { tail -5 gpurun_out/${tag}_gpmc.log; exit 1; }
ls gpurun_out/${tag}_gpmc
