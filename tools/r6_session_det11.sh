set -o pipefail
for kv in "DLAP_WIDE=1 DLAP_PP_GLOBAL=1"; do
  for i in 1 2 3 4; do echo "== $kv ($i)"; timeout -k 10 300 env $kv python3 tools/wide_det_probe2.py 2>&1 | grep -v amdgpu.ids | tail -2 | cut -c1-200 || exit 1; done; done
