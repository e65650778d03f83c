# G=2 epoch: kernel trace timeline (steady phase 3)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6t}
$T 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 --models-per-gpu 2 > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/${tag}_prof --adams 2 --marker k_begin_phase > gpurun_out/${tag}_timeline.txt || true
rm -rf gpurun_out/${tag}_prof
wc -l gpurun_out/${tag}_timeline.txt
