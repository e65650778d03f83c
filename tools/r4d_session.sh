bash tools/r4_ab.sh r4d \
 "s_c1|DLAP_GRAPH_COPIES=1|--steps 20 --warmup 5 --no-ensemble9" \
 "s_c3|DLAP_GRAPH_COPIES=3|--steps 20 --warmup 5 --no-ensemble9" \
 "l_c1|DLAP_GRAPH_COPIES=1|--steps 210 --warmup 21 --no-ensemble9" \
 "l_c3|DLAP_GRAPH_COPIES=3|--steps 210 --warmup 21 --no-ensemble9" \
 "g9_f4|DLAP_BWD_FPW=4|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
 "g9_f1|DLAP_BWD_FPW=1|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
 "g9_cap|DLAP_FUSED_CAP=4096|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
 "g9_nof|DLAP_RNN_OVERLAP=0|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
 "g9_nop|DLAP_GRAM_PLAN=0|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" && \
bash tools/r4_hiptrace.sh r4dh DLAP_GRAPH_COPIES=3 && \
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -s --timeout 280 --timeout-method thread > gpurun_out/r4d_parity.log 2>&1; tail -8 gpurun_out/r4d_parity.log
