# epoch timeline of the current tree (kernel trace of a 60-step bench run)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6d}
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/${tag}_prof --adams 3 --marker k_lstm_tail > gpurun_out/${tag}_timeline.txt || true
python3 tools/kernel_stats.py gpurun_out/${tag}_prof > gpurun_out/${tag}_kernel_stats.txt 2>&1 || true
head -50 gpurun_out/${tag}_timeline.txt
