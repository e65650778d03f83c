#!/bin/bash
# GPU suite inside the host-ASan harness (the runtime's host code instrumented; device code not).
# Deselected: the in-tree .so location check (the engine is a built-in module here). The 2-rank
# spawn test's children re-run sys.executable = this harness with "-c" (supported).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# torch dlopens some of its libraries by bare name; the python binary finds them, the harness
# executable needs torch/lib on the search path
TORCH_LIB=$(python3 -c "import importlib.util, os; print(os.path.join(os.path.dirname(importlib.util.find_spec('torch').origin), 'lib'))")
export LD_LIBRARY_PATH="$TORCH_LIB${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}"
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 DLAP_CRASH_TRACE=0 PYTHONHOME=/usr \
  timeout -k 10 600 ./deeplearninginassetpricing_paperreplication_amd/asan/dlap_asan_python tools/asan_pytest.py \
  tests -m gpu -x -q -p no:cacheprovider --deselect tests/test_engine_gpu.py::test_extension_is_native --timeout 300 --timeout-method thread > gpurun_out/asan_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/asan_gpu_tests.log
exit $rc
