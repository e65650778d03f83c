# row-proportional grids of the streamed (wide) forwards: wide-path tests, scaled bench + kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6w}
rc=0
$T 600 python -u -m pytest --maxfail=5 -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_engine_fp32_gpu.py tests/test_dropout_gpu.py -k "wide or F200 or forced" > gpurun_out/${tag}_tests.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/${tag}_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
$T 400 python bench.py --config scaled --steps 20 --warmup 5 > gpurun_out/${tag}_scaled.log 2>&1 || { tail -20 gpurun_out/${tag}_scaled.log; exit 1; }
tail -1 gpurun_out/${tag}_scaled.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]' | tr '\n' ' '; echo
$T 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_sprof -o run -- python3 bench.py --config scaled --steps 10 --warmup 3 > gpurun_out/${tag}_sprof.log 2>&1 || { tail -5 gpurun_out/${tag}_sprof.log; exit 1; }
python3 tools/kernel_stats.py gpurun_out/${tag}_sprof > gpurun_out/${tag}_scaled_kernels.txt 2>&1 || true
rm -rf gpurun_out/${tag}_sprof
grep "k_mlp\|k_wgrad\|k_gram\|k_proj0\|k_lstm_tail\|k_period" gpurun_out/${tag}_scaled_kernels.txt | cut -c1-110
