# one-pass backward at HL = 4: equality with the sliced kernel, HL4 bucket costs A/B
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6x}
rc=0
$T 600 python -u -m pytest --maxfail=5 -v --timeout 300 --timeout-method thread tests/test_tbwd_gpu.py > gpurun_out/${tag}_tests.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
for v in 0 1; do
  DLAP_TBWD4=$v $T 300 python -u tools/sweep_costs.py --grid paper --only HL4-H4-CH0 --epochs 12 --out gpurun_out/${tag}_c$v.json > gpurun_out/${tag}_c$v.log 2>&1 || { tail -20 gpurun_out/${tag}_c$v.log; exit 1; }
  echo "TBWD4=$v"; grep ms/epoch gpurun_out/${tag}_c$v.log
done
