set -o pipefail
for i in 1 2; do timeout -k 10 300 env DLAP_WIDE=1 python3 tools/wide_det_probe2.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1; done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gram_gpu.py tests/test_invariance_gpu.py tests/test_engine_gpu.py tests/test_engine_fp32_gpu.py > gpurun_out/r6det8_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6det8_tests.log; exit $rc
