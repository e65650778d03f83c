#!/bin/bash
# Round-5 session 14: split epoch graphs (chain | evaluation, in-kernel hand-offs) -- tests, A/B, timeline
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_invariance_gpu.py > gpurun_out/r5_s14_t1.log 2>&1 || { tail -40 gpurun_out/r5_s14_t1.log; exit 1; }
tail -2 gpurun_out/r5_s14_t1.log
OUT=gpurun_out/r5_s14_bench.log; : > $OUT
b() { local tag=$1; shift; local a="$1"; shift
  line=$($T 200 env "$@" python3 bench.py $a --no-ensemble9 2>>gpurun_out/r5_s14.err | tail -1) || { echo "[$tag] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$tag] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT; }
L="--steps 210 --warmup 21"
b long_split "$L"
b long_kadam "$L" DLAP_TAIL_ADAM=0
b short_split "--steps 20 --warmup 5"
b short_kadam "--steps 20 --warmup 5" DLAP_TAIL_ADAM=0
b long_split2 "$L"
b long_kadam2 "$L" DLAP_TAIL_ADAM=0
b g2 "--steps 60 --warmup 10 --models-per-gpu 2"
cat $OUT
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace -d gpurun_out/r5_s14_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/r5_s14_prof.log 2>&1 || { tail -5 gpurun_out/r5_s14_prof.log; exit 1; }
python3 tools/run_timeline.py gpurun_out/r5_s14_prof --adams 3 --marker k_lstm_tail > gpurun_out/r5_s14_timeline.txt || true
head -40 gpurun_out/r5_s14_timeline.txt
