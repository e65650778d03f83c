#!/bin/bash
# Round-4 session G: the fpw>1 backward (weights staged once, fine + coarse images in LDS), the
# compile-time one-slab SDF backward and the TPS=1 / two-waves default: invariance, then timing.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_invariance_gpu.py > gpurun_out/r4g_inv.log 2>&1 \
  || { echo "invariance FAILED"; tail -30 gpurun_out/r4g_inv.log; exit 3; }
grep -E "PASSED|FAILED" gpurun_out/r4g_inv.log
bash tools/r4_ab.sh r4g \
  "l_def||--steps 210 --warmup 21 --no-ensemble9" \
  "l_tps2|DLAP_TPS=2|--steps 210 --warmup 21 --no-ensemble9" \
  "s_def||--steps 20 --warmup 5 --no-ensemble9" \
  "g9_def||--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
  "g9_f1|DLAP_BWD_FPW=1|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
  "g3_def||--models-per-gpu 3 --steps 100 --warmup 10 --no-ensemble9" \
  "g3_f1|DLAP_BWD_FPW=1|--models-per-gpu 3 --steps 100 --warmup 10 --no-ensemble9" \
  "g9_c16|DLAP_BWD_FPW=1 DLAP_NSLAB_COARSE=16|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" && \
bash tools/r4_kstats.sh r4gk9 "" --models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9
