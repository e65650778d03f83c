#!/bin/bash
# Driver-argument bench (--steps 20 --warmup 5, or $BARGS) under engine knobs (env), R repeats
# each; one line per run in gpurun_out/knobs_short.log.
# Usage (GPU box): R=2 bash tools/knobs_short.sh "" "DLAP_TRAIN_FIRST=2" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
BARGS=${BARGS:-"--steps 20 --warmup 5"}
R=${R:-1}
for kv in "$@"; do
  for r in $(seq $R); do
    out=$(env $kv timeout -k 10 150 python -u bench.py $BARGS --no-ensemble9 2>/dev/null)
    rc=$?
    echo "[$kv] rc=$rc $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["ms_per_epoch_phase"])' 2>&1)" | tee -a gpurun_out/knobs_short.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
