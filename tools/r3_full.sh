#!/bin/bash
# GPU suite + driver-argument bench + long bench (r3_round.sh), then the kernel-trace timeline of
# the driver-argument bench (r3_prof_short.sh). Usage: bash tools/r3_full.sh <tag>
set -o pipefail
TAG=${1:-fu}
bash tools/r3_round.sh ${TAG} || exit $?
bash tools/r3_prof_short.sh ${TAG}p
