#!/bin/bash
# HBM bytes per kernel (FETCH_SIZE, WRITE_SIZE: two passes, TCC counter limits) of a bench config.
# Usage (GPU box): bash tools/r4_pmc_bytes.sh <tag> <bench args...>
TAG=$1; shift
cd /tmp || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_f -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/${TAG}_f.log 2>&1 || exit 5
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_w -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/${TAG}_w.log 2>&1 || exit 6
python3 $R/tools/pmc_bytes_table.py $R/gpurun_out/${TAG}_f $R/gpurun_out/${TAG}_w > $R/gpurun_out/${TAG}_bytes.txt
rm -rf $R/gpurun_out/${TAG}_f $R/gpurun_out/${TAG}_w
cat $R/gpurun_out/${TAG}_bytes.txt | head -30
