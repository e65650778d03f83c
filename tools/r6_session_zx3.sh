# streamed wide forward with the three-slot unrolled chunk loop: wide-path tests, scaled bench, kernel table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6zx3}
rc=0
$T 600 python -u -m pytest --maxfail=3 -v --timeout 300 --timeout-method thread tests/test_tbwd_gpu.py tests/test_dropout_gpu.py tests/test_engine_gpu.py -k "wide" > gpurun_out/${tag}_tests.log 2>&1 || rc=$?
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/${tag}_tests.log | tail -12
[ $rc -eq 0 ] || exit 1
bash tools/scaled_knobs.sh ${tag}_k - || exit 1
$T 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${tag}_sprof -o run -- python3 bench.py --config scaled --steps 10 --warmup 3 > gpurun_out/${tag}_sprof.log 2>&1 || { tail -5 gpurun_out/${tag}_sprof.log; exit 1; }
python3 tools/kernel_stats.py gpurun_out/${tag}_sprof > gpurun_out/${tag}_scaled_kernels.txt 2>&1 || true
python3 tools/run_timeline.py gpurun_out/${tag}_sprof --adams 3 --marker k_lstm_tail > gpurun_out/${tag}_scaled_timeline.txt 2>&1 || true
rm -rf gpurun_out/${tag}_sprof
grep -E "k_tbwd|k_mlp_fwd_zx|k_wgrad0|k_period" gpurun_out/${tag}_scaled_kernels.txt
