#!/bin/bash
# Bench the real config under engine launch knobs (env); one line per setting in
# gpurun_out/knobs.log. Usage (GPU box): bash tools/knob_sweep.sh "DLAP_GX_FWD=512" "DLAP_PRIO=1" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "" "$@"; do
  out=$(env $kv timeout -k 10 120 python -u bench.py --no-ensemble9 2>/dev/null)
  rc=$?
  echo "[$kv] rc=$rc $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_epoch_phase"])' 2>&1)" | tee -a gpurun_out/knobs.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
