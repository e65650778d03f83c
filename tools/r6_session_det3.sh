set -o pipefail
mkdir -p gpurun_out
for kv in "DLAP_WIDE=1" "DLAP_WIDE=1 DLAP_ZX_EVAL=0" "DLAP_WIDE=1 DLAP_ZX_TRAIN=0" "DLAP_WIDE=0"; do
  echo "== $kv"; timeout -k 10 300 env $kv python3 tools/wide_det_probe2.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1; done
