# cheaper dropout hash, train Gram beside the head forward: tests, bench A/B, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6m}
rc=0
$T 600 python -u -m pytest --maxfail=5 -v --timeout 300 --timeout-method thread tests/test_gram_gpu.py \
  tests/test_invariance_gpu.py -k "train_gram or split_epoch or adam_in_tail" > gpurun_out/${tag}_tests.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
for side in 0 1; do
for a in "--steps 20 --warmup 5" "--steps 210 --warmup 21"; do
  DLAP_TRAIN_GRAM_SIDE=$side $T 300 python bench.py $a --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  echo "side=$side $a $(tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' ')"
done
done
DLAP_TRAIN_GRAM_SIDE=1 $T 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/${tag}_prof.log 2>&1 || { tail -5 gpurun_out/${tag}_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/${tag}_prof --adams 2 --marker k_begin_phase > gpurun_out/${tag}_timeline.txt || true
grep -m3 k_dropmask gpurun_out/${tag}_timeline.txt
