set -o pipefail
for i in 1 2; do timeout -k 10 300 env DLAP_WIDE=1 python3 tools/wide_det_probe2.py 4 2>&1 | grep -v amdgpu.ids | tail -4 | cut -c1-200 || exit 1; done
