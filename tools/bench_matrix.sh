#!/bin/bash
# The driver's bench line (with the ensemble) and the other BASELINE configs on one GPU.
# Usage: gpurun --timeout 1200 -- bash tools/bench_matrix.sh <tag>
set -o pipefail
tag=${1:-matrix}
mkdir -p gpurun_out
OUT=gpurun_out/${tag}.log; : > $OUT
run() { local name=$1; shift
  echo "== $name: bench.py $*" >> $OUT
  timeout -k 10 400 python3 bench.py "$@" 2>>gpurun_out/${tag}.err | tail -1 | cut -c1-1500 >> $OUT || { echo "[$name] FAILED" >> $OUT; cat $OUT; exit 1; }
}
run driver_short --steps 20 --warmup 5
run default
run g9 --models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9
run scaled --config scaled --steps 20 --warmup 5 --no-ensemble9
cat $OUT
