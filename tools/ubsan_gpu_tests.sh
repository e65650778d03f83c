#!/bin/bash
# Run the GPU test suite against a checking build of the native extension:
#   ubsan (default): host UBSan in trap mode;   debug: device-side bounds assertions.
# Build it first on the CPU side:
#   python -m deeplearninginassetpricing_paperreplication_amd.engine.build --ubsan   (or --debug)
# Usage on the GPU box: bash tools/ubsan_gpu_tests.sh [ubsan|debug] [pytest -k expression]
set -u
VARIANT=${1:-ubsan}
SEL=${2:-}
export DLAP_NATIVE=$VARIANT DLAP_AUTOBUILD=0
if [ -n "$SEL" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$SEL"
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
rc=$?
echo "$VARIANT gpu tests rc=$rc"
exit $rc
