# eval recurrences on the eval queue, fused tail for stacked H=4 layers, safe-mode fallback; bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6i}
rc=0
$T 900 python -u -m pytest --maxfail=10 -v --timeout 300 --timeout-method thread \
  tests/test_invariance_gpu.py -k "other_lstm or phase2_tail or eval_queue or safe_mode or poisons or split_epoch or adam_in_tail or handoff or concurrent or eval_recurrences" \
  "tests/test_engine_fp32_gpu.py::test_fp32_trajectory_matches_cpu_trainer[paper_cm32]" \
  > gpurun_out/${tag}_tests.log 2>&1 || rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -30
[ $rc -le 1 ] || exit $rc
for a in "--steps 210 --warmup 21" "--steps 20 --warmup 5"; do
  $T 300 python bench.py $a --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench.log | cut -c1-300; tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_epoch_phase[^]]*]'
done
$T 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/${tag}_prof --adams 2 --marker k_begin_phase > gpurun_out/${tag}_timeline.txt || true
wc -l gpurun_out/${tag}_timeline.txt
