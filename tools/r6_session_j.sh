# full GPU suite, driver-argument and steady bench, kernel-trace timeline of the short run
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6j}
rc=0
$T 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${tag}_suite.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_suite.log | tail -20
[ $rc -le 1 ] || exit $rc
for a in "--steps 20 --warmup 5" "--steps 210 --warmup 21"; do
  $T 300 python bench.py $a --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]'
done
$T 300 python bench.py > gpurun_out/${tag}_bench_default.log 2>&1 || { tail -20 gpurun_out/${tag}_bench_default.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_default.log | cut -c1-200
