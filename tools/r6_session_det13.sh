set -o pipefail
for i in 1 2 3; do echo "== DLAP_ZX_EVAL_SPLIT=1 ($i)"; timeout -k 10 300 env DLAP_WIDE=1 DLAP_ZX_EVAL_SPLIT=1 python3 tools/wide_det_probe2.py 2>&1 | grep -v amdgpu.ids | tail -2 | cut -c1-200 || exit 1; done
