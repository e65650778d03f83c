# new GPU tests (xs engine, generalized fused tail, paper-grid fp32 branches, sweep slice), xs
# timings, G=1 vs G=2 epoch
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6h}
rc=0
$T 900 python -u -m pytest --maxfail=8 -v --timeout 300 --timeout-method thread tests/test_xsection_gpu.py \
  "tests/test_invariance_gpu.py::test_fused_backward_tail_other_lstm_shapes" \
  "tests/test_invariance_gpu.py::test_fused_backward_tail_equals_separate_kernels" "tests/test_invariance_gpu.py::test_phase2_tail_and_lstm_once_equal_separate_kernels" "tests/test_invariance_gpu.py::test_wait_give_up_falls_back_to_safe_mode" "tests/test_invariance_gpu.py::test_fused_wait_give_up_poisons_the_model" \
  tests/test_engine_fp32_gpu.py -k "paper or default or xsection or sweep or tail" tests/test_sweep_gpu.py \
  > gpurun_out/${tag}_tests.log 2>&1 || rc=$?
tail -30 gpurun_out/${tag}_tests.log
# (plain test failures, rc 1, still measure; anything else -- a fault, abort or time limit -- stops)
[ $rc -le 1 ] || exit $rc
$T 300 python -u tools/xs_bench.py > gpurun_out/${tag}_xs1.log 2>&1 || { tail -30 gpurun_out/${tag}_xs1.log; exit 1; }
tail -2 gpurun_out/${tag}_xs1.log
DLAP_SHARE_GPU=1 DLAP_DIST_BACKEND=gloo $T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/xs_bench.py > gpurun_out/${tag}_xs2.log 2>&1 || { tail -30 gpurun_out/${tag}_xs2.log; exit 1; }
tail -2 gpurun_out/${tag}_xs2.log
for G in 1 2; do
  $T 300 python bench.py --steps 210 --warmup 21 --no-ensemble9 --models-per-gpu $G > gpurun_out/${tag}_g$G.log 2>&1 || { tail -20 gpurun_out/${tag}_g$G.log; exit 1; }
  tail -1 gpurun_out/${tag}_g$G.log | cut -c1-400
done
