#!/bin/bash
# Multi-rank rehearsal on ONE GPU (gloo, ranks share the device): bench.py at 2 and 4 ranks;
# the ensemble9 member trajectories must not depend on the sharding, so the ensemble test /
# valid Sharpe must equal the 1-rank bench's (tools/r4_check.sh <tag>_short*.log).
set -o pipefail
TAG=${1:-rh}
mkdir -p gpurun_out
export TMPDIR=/tmp DLAP_DIST_BACKEND=gloo DLAP_SHARE_GPU=1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_n1.log 2>&1 || { tail -20 gpurun_out/${TAG}_n1.log; exit 3; }
grep -o '"test_sharpe": [0-9.-]*\|"valid_sharpe": [0-9.-]*\|"panel_setup_s": [0-9.]*\|"fused_wait_timeouts": [0-9]*' gpurun_out/${TAG}_n1.log | tr '\n' ' '; echo
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/${TAG}_n$n.log 2>&1 || { tail -20 gpurun_out/${TAG}_n$n.log; exit 3; }
  grep -o '"test_sharpe": [0-9.-]*\|"valid_sharpe": [0-9.-]*\|"panel_setup_s_rank0": [0-9.]*\|"fused_wait_timeouts": [0-9]*\|"models_per_rank": \[[^]]*\]' gpurun_out/${TAG}_n$n.log | tr '\n' ' '; echo
done
