set -o pipefail
mkdir -p gpurun_out
echo "== DLAP_WIDE=1"
timeout -k 10 200 env DLAP_WIDE=1 python3 tools/wide_det_probe.py 2>&1 | tail -30 || exit 1
bash tools/scaled_knobs.sh r6det2_k - || exit 1
