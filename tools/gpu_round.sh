#!/bin/bash
# Run GPU steps "name:timeout_s:command" in order; logs go to gpurun_out/<name>.log.
# A normal failure (exit 1, e.g. a failed check) continues; any abnormal exit (timeout,
# abort, segfault, GPU fault) stops the round so nothing else touches the GPU.
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "== $name (limit ${to}s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "rc=$rc" >> "gpurun_out/$name.log"
  echo "   rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after abnormal exit $rc"; exit $rc; fi
done
