# final evidence on the round-6 tree: GPU suite, smoke, benches (default, short, scaled), kernel stats + timeline, xsection CLI
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6fin}
rc=0
$T 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${tag}_suite.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_suite.log | tail -8
[ $rc -le 1 ] || exit $rc
$T 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -20 gpurun_out/${tag}_smoke.log; exit 1; }
tail -1 gpurun_out/${tag}_smoke.log
$T 400 python bench.py > gpurun_out/${tag}_bench_default.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_default.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_default.log | cut -c1-260; echo
grep -o '"ensemble9": {[^}]*' gpurun_out/${tag}_bench_default.log | cut -c1-300
$T 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench_short.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_short.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_short.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' '; echo
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/${tag}_prof --adams 2 --marker k_begin_phase > gpurun_out/${tag}_timeline.txt || true
python3 tools/kernel_stats.py gpurun_out/${tag}_prof > gpurun_out/${tag}_kernel_stats.txt 2>&1 || true
rm -rf gpurun_out/${tag}_prof
head -12 gpurun_out/${tag}_kernel_stats.txt
$T 300 python -m deeplearninginassetpricing_paperreplication_amd.parallel.xsection --synthetic 240 60 300 3000 46 178 --epochs 16 4 16 --ignore_epoch 2 --print_freq 8 > gpurun_out/${tag}_xs_cli.log 2>&1 || { tail -20 gpurun_out/${tag}_xs_cli.log; exit 1; }
tail -1 gpurun_out/${tag}_xs_cli.log
$T 400 python bench.py --config scaled --steps 20 --warmup 5 > gpurun_out/${tag}_bench_scaled.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_scaled.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_scaled.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' '; echo
