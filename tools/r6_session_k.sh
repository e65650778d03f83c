# K=32 fp32 trajectory triage under engine switches; bench
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6k}
: > gpurun_out/${tag}_probe.log
for env in "" "DLAP_SPLIT_GRAPHS=0" "DLAP_SPLIT_GRAPHS=0 DLAP_TAIL_ADAM=0" "DLAP_GRAM=0" "DLAP_FUSED_TAIL=0" "DLAP_RNN_OVERLAP=0" "DLAP_H_CACHE=0"; do
  $T 120 python tools/traj_probe.py '{"num_condition_moment": 32}' $env >> gpurun_out/${tag}_probe.log 2>&1 || { tail -20 gpurun_out/${tag}_probe.log; exit 1; }
done
$T 120 python tools/traj_probe.py '{}' >> gpurun_out/${tag}_probe.log 2>&1 || exit 1
grep '^{' gpurun_out/${tag}_probe.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['env'], 'gn', ['%.1e' % x for x in d['rel_gn']], 'worst', {k: '%.1e' % v for k, v in d['worst'].items()}, d['info'])"
for a in "--steps 20 --warmup 5" "--steps 210 --warmup 21"; do
  $T 300 python bench.py $a --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench.log | grep -o '"ms_per_step": [0-9.]*\|"ms_per_epoch_phase": \[[^]]*\]'
done
