#!/bin/bash
# 1 / 2 / 4-rank rehearsal on ONE GPU (gpurun box): the bench and the 9-seed ensemble trainer under
# torch.distributed.run, gloo collectives, every rank on GPU 0 (DLAP_SHARE_GPU=1). The ensemble's
# test Sharpe must not depend on the rank count (members are bitwise invariant to sharding).
# Usage: gpurun --timeout 1200 -- bash tools/rehearse_multirank.sh
set -o pipefail
mkdir -p gpurun_out
export DLAP_DIST_BACKEND=gloo DLAP_SHARE_GPU=1
OUT=gpurun_out/rehearsal.log; : > $OUT
run() { local name=$1 to=$2; shift 2
  echo "== $name: $*" >> $OUT
  timeout -k 10 "$to" "$@" > gpurun_out/rehearsal_$name.log 2>&1 || { echo "[$name] FAILED rc=$?" >> $OUT; tail -20 gpurun_out/rehearsal_$name.log; cat $OUT; exit 1; }
  tail -2 gpurun_out/rehearsal_$name.log | cut -c1-600 >> $OUT; }
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
ENS="-m deeplearninginassetpricing_paperreplication_amd.parallel.ensemble --synthetic 240 60 300 3000 46 178 --epochs_unc 32 --epochs_moment 8 --epochs 64 --ignore_epoch 4"
run bench_n2 300 $TR --nproc-per-node 2 --master-port 29511 bench.py --gpus 2 --steps 105 --warmup 12
run bench_n4 300 $TR --nproc-per-node 4 --master-port 29512 bench.py --gpus 4 --steps 105 --warmup 12
run ens_n1 300 $TR --nproc-per-node 1 --master-port 29513 $ENS
run ens_n2 300 $TR --nproc-per-node 2 --master-port 29514 $ENS
run ens_n4 300 $TR --nproc-per-node 4 --master-port 29515 $ENS
cat $OUT
