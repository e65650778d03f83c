set -o pipefail
mkdir -p gpurun_out
for kv in "DLAP_WIDE=1" "DLAP_WIDE=1 DLAP_ZX_EVAL=0" "DLAP_WIDE=1 DLAP_SPLIT_GRAPHS=0"; do
  echo "== $kv"
  timeout -k 10 200 env $kv python3 tools/wide_det_probe.py 2>&1 | tail -30 || exit 1
done
