# A/B of engine knobs on the scaled panel (config 5). Usage:
#   gpurun -- bash tools/scaled_knobs.sh <tag> "NAME=V ..." ...   ("-" = defaults)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
OUT=gpurun_out/${tag}.log; : > $OUT
for arm in "$@"; do
  kv=$arm; [ "$arm" = "-" ] && kv="X_DEFAULT=1"
  line=$(timeout -k 10 300 env $kv python3 bench.py --config scaled --steps 20 --warmup 5 2>>gpurun_out/${tag}.err | tail -1) || { echo "[$arm] FAILED" >> $OUT; cat $OUT; exit 1; }
  echo "[$arm] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_epoch_phase"])')" >> $OUT
done
cat $OUT
