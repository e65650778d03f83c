#!/bin/bash
# A/B runs of the bench under environment knobs. Each line: "<tag>|<env...>|<bench args>".
# Usage (GPU box): bash tools/r4_ab.sh <prefix> "<tag>|<env>|<args>" ...
set -o pipefail
P=${1:-ab}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r tag envs args <<< "$spec"
  env $envs timeout -k 10 200 python -u bench.py $args > gpurun_out/${P}_${tag}.log 2>&1 || { echo "[$tag] FAILED"; tail -20 gpurun_out/${P}_${tag}.log; exit 3; }
  echo "[$tag] $envs $args :: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]\|"wall_s": [0-9.]*\|"epochs": [0-9.]*\|"train_total": [0-9.]*' gpurun_out/${P}_${tag}.log | tr '\n' ' ')"
done
