#!/bin/bash
# Round-5 session 17: stream priorities with the split epoch graphs
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
OUT=gpurun_out/r5_s17_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s17.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"], "host", d["host_enqueue_ms_per_step"], d["host_launch_us_per_epoch"])')" >> $OUT; }
L="--steps 210 --warmup 21"
b long_split "$L"
b long_split_prio "$L" DLAP_PRIO=1
b short_split "--steps 20 --warmup 5"
b short_split_prio "--steps 20 --warmup 5" DLAP_PRIO=1
b long_split2 "$L"
b long_split_prio2 "$L" DLAP_PRIO=1
b g2_prio "--steps 60 --warmup 10 --models-per-gpu 2" DLAP_PRIO=1
cat $OUT
export TMPDIR=/tmp
timeout -k 10 300 env DLAP_PRIO=1 rocprofv3 --kernel-trace -d gpurun_out/r5_s17_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/r5_s17_prof.log 2>&1 || { tail -5 gpurun_out/r5_s17_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/r5_s17_prof --adams 3 --marker k_lstm_tail > gpurun_out/r5_s17_timeline.txt || true
sed -n 10,30p gpurun_out/r5_s17_timeline.txt
