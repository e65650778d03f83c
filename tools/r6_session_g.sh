# cross-sectional engine path: GPU tests, 1-rank and 2-rank (shared GPU) epoch timings
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6g}
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xsection_gpu.py > gpurun_out/${tag}_tests.log 2>&1 || { tail -60 gpurun_out/${tag}_tests.log; exit 1; }
tail -12 gpurun_out/${tag}_tests.log
$T 300 python -u tools/xs_bench.py > gpurun_out/${tag}_xs1.log 2>&1 || { tail -30 gpurun_out/${tag}_xs1.log; exit 1; }
tail -2 gpurun_out/${tag}_xs1.log
DLAP_SHARE_GPU=1 DLAP_DIST_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/xs_bench.py > gpurun_out/${tag}_xs2.log 2>&1 || { tail -30 gpurun_out/${tag}_xs2.log; exit 1; }
tail -2 gpurun_out/${tag}_xs2.log
