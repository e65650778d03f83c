#!/bin/bash
# bench phase timings for several MLP grid sizes (sequential epoch graph for clean numbers)
for f in 256 512 1024 2048 4096; do
  echo "GX_FWD=$f"; DLAP_PIPELINE=0 DLAP_GX_FWD=$f timeout -k 10 120 python3 bench.py --steps 63 --warmup 9 | grep -o '"ms_per_epoch_phase": \[[^]]*\]' || exit $?
done
for b in 128 256 512 1024; do
  echo "GX_BWD=$b"; DLAP_PIPELINE=0 DLAP_GX_BWD=$b timeout -k 10 120 python3 bench.py --steps 63 --warmup 9 | grep -o '"ms_per_epoch_phase": \[[^]]*\]' || exit $?
done
