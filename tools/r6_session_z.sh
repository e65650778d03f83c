# one-pass backward on the wide path: equality tests, scaled-panel A/B against the sliced kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6z}
rc=0
$T 600 python -u -m pytest --maxfail=3 -v --timeout 300 --timeout-method thread tests/test_tbwd_gpu.py tests/test_dropout_gpu.py -k "wide or one_pass" > gpurun_out/${tag}_tests.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/${tag}_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
for v in 1 0; do
  DLAP_TBWD=$v $T 400 python bench.py --config scaled --steps 20 --warmup 5 > gpurun_out/${tag}_tb$v.log 2>&1 || { tail -20 gpurun_out/${tag}_tb$v.log; exit 1; }
  echo "TBWD=$v"; tail -1 gpurun_out/${tag}_tb$v.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' '; echo
done
$T 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_sprof -o run -- python3 bench.py --config scaled --steps 10 --warmup 3 > gpurun_out/${tag}_sprof.log 2>&1 || { tail -5 gpurun_out/${tag}_sprof.log; exit 1; }
python3 tools/kernel_stats.py gpurun_out/${tag}_sprof > gpurun_out/${tag}_scaled_kernels.txt 2>&1 || true
python3 tools/run_timeline.py gpurun_out/${tag}_sprof --adams 3 --marker k_lstm_tail > gpurun_out/${tag}_scaled_timeline.txt 2>&1 || true
grep -E "k_tbwd|k_mlp_fwd_zx|k_wgrad0|k_period" gpurun_out/${tag}_scaled_kernels.txt
