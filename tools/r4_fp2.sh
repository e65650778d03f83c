#!/bin/bash
# Full GPU suite + smoke + default bench (r4_full_gpu.sh), then two driver-argument short runs and
# the short-run kernel trace.
set -o pipefail
bash tools/r4_full_gpu.sh || exit $?
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r4_fp2_short$i.log 2>&1 || { tail -20 gpurun_out/r4_fp2_short$i.log; exit 5; }
  tail -1 gpurun_out/r4_fp2_short$i.log | cut -c1-220
done
bash tools/r3_prof_short.sh r4fp2 > gpurun_out/r4fp2_prof_summary.txt 2>&1 || exit 7
