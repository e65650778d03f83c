#!/bin/bash
# Round-5 session 9: epoch timelines of the rotated pipeline and of the chain without the evaluation branch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for arm in rot:DLAP_ROTATE=1 noeval:DLAP_SKIP=2; do
  tag=${arm%%:*}; kv=${arm#*:}
  export $kv
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r5_s9_$tag -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/r5_s9_$tag.log 2>&1 || { tail -20 gpurun_out/r5_s9_$tag.log; exit 1; }
  unset ${kv%%=*}
  python3 tools/run_timeline.py gpurun_out/r5_s9_$tag --adams 3 > gpurun_out/r5_s9_timeline_$tag.txt
  echo "== $tag"; head -30 gpurun_out/r5_s9_timeline_$tag.txt
done
