set -o pipefail
for i in 1 2; do echo "== old streamed forward, DLAP_WIDE=1 run $i"; timeout -k 10 300 env DLAP_WIDE=1 python3 tools/wide_det_probe2.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1; done
