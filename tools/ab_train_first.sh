#!/bin/bash
# A/B of the epoch-graph capture order (DLAP_TRAIN_FIRST), then a kernel-trace timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/knobs.log
bash tools/knob_sweep.sh DLAP_TRAIN_FIRST=0 DLAP_TRAIN_FIRST=1 DLAP_TRAIN_FIRST=0 DLAP_TRAIN_FIRST=1 DLAP_TRAIN_FIRST=0 DLAP_TRAIN_FIRST=1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tf -o prof -- python3 bench.py --no-ensemble9 > gpurun_out/ab_prof.log 2>&1
