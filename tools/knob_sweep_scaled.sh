#!/bin/bash
# knob_sweep.sh for the scaled panel (600 x 30000 x 512, wide layer-0 path).
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in "" "$@"; do
  out=$(env $kv timeout -k 10 300 python -u bench.py --config scaled --steps 42 --warmup 6 2>/dev/null)
  rc=$?
  echo "[$kv] rc=$rc $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_epoch_phase"])' 2>&1)" | tee -a gpurun_out/knobs_scaled.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
