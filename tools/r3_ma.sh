#!/bin/bash
# Module-API / ensemble / xsection GPU tests (failures do not stop the profile), then the
# driver-argument bench under a kernel trace (tools/r3_prof_short.sh).
set -o pipefail
TAG=${1:-ma}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_module_autograd_gpu.py tests/test_engine_gpu.py tests/test_xsection_gpu.py \
    -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -40 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
bash tools/r3_prof_short.sh ps1
