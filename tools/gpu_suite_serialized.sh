#!/bin/bash
# GPU suite with every kernel launch serialised (a fault is reported at the launch that caused
# it), then the normal suite.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ser_gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/ab_gpu_tests2.log 2>&1
