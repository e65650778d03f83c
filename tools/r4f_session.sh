#!/bin/bash
set -o pipefail
bash tools/r4_ab.sh r4f \
 "l_base||--steps 210 --warmup 21 --no-ensemble9" \
 "l_bwd1|DLAP_NATIVE=bwd1 DLAP_BWD_FPW=1|--steps 210 --warmup 21 --no-ensemble9" \
 "l_tps1|DLAP_TPS=1|--steps 210 --warmup 21 --no-ensemble9" \
 "l_wps2|DLAP_NATIVE=wps2 DLAP_TPS=1|--steps 210 --warmup 21 --no-ensemble9" \
 "l_u8|DLAP_UNROLL=8|--steps 210 --warmup 21 --no-ensemble9" \
 "s_base||--steps 20 --warmup 5 --no-ensemble9" \
 "s_u8|DLAP_UNROLL=8|--steps 20 --warmup 5 --no-ensemble9" \
 "l_pc0|DEBUG_CLR_GRAPH_PACKET_CAPTURE=0|--steps 210 --warmup 21 --no-ensemble9" \
 "g9_f1|DLAP_BWD_FPW=1|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
 "g9_bwd1|DLAP_NATIVE=bwd1 DLAP_BWD_FPW=1|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" \
 "g9_c16|DLAP_BWD_FPW=1 DLAP_NSLAB_COARSE=16|--models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9" && \
bash tools/r4_kstats.sh r4fk9 "DLAP_BWD_FPW=1" --models-per-gpu 9 --steps 60 --warmup 10 --no-ensemble9 && \
bash tools/r4_kstats.sh r4fk1 "" --steps 210 --warmup 21 --no-ensemble9
