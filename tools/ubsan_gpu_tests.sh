#!/bin/bash
# Run the GPU test suite against the host-UBSan (trap mode) build of the native extension.
# Build it first on the CPU side:  python -m deeplearninginassetpricing_paperreplication_amd.engine.build --ubsan
# Usage on the GPU box: bash tools/ubsan_gpu_tests.sh   (restores the normal .so afterwards)
set -u
PKG=deeplearninginassetpricing_paperreplication_amd
SO=$(ls $PKG/_dlap_hip*.so)
cp "$SO" /tmp/_dlap_hip_normal.so || exit 1
cp $PKG/ubsan/$(basename "$SO") "$SO" || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
rc=$?
cp /tmp/_dlap_hip_normal.so "$SO"
echo "ubsan gpu tests rc=$rc"
exit $rc
