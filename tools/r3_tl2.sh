#!/bin/bash
# Short-run kernel timelines for two engine settings (A/B). Usage: bash tools/r3_tl2.sh <tag> "<envA>" "<envB>"
set -o pipefail
TAG=${1:-tl}
bash tools/r3_prof_short.sh ${TAG}a $2 > gpurun_out/${TAG}a.out 2>&1 || { tail -5 gpurun_out/${TAG}a.out; exit 3; }
head -3 gpurun_out/${TAG}a.out
bash tools/r3_prof_short.sh ${TAG}b $3 > gpurun_out/${TAG}b.out 2>&1 || { tail -5 gpurun_out/${TAG}b.out; exit 4; }
head -3 gpurun_out/${TAG}b.out
