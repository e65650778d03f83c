# in-kernel timing of the fused forward / tail, and the short-run kernel trace on the current tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6l}
$T 200 python tools/lstm_timing.py > gpurun_out/${tag}_lstm_timing.log 2>&1 || { tail -20 gpurun_out/${tag}_lstm_timing.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_lstm_timing.log
$T 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/${tag}_prof --adams 2 --marker k_begin_phase > gpurun_out/${tag}_timeline.txt || true
wc -l gpurun_out/${tag}_timeline.txt
