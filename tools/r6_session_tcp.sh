# TCP / UTCL1 counters of the scaled-panel kernels (address translation, L2 requests)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r6tcp}
timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d gpurun_out/${tag}_p1 -o run -- python3 bench.py --config scaled --steps 4 --warmup 1 > gpurun_out/${tag}_p1.log 2>&1 || { tail -5 gpurun_out/${tag}_p1.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/${tag}_p1 > gpurun_out/${tag}_pmc.txt 2>&1 || true
grep -A6 "k_mlp_fwd_zx\|k_wgrad0<PrecBF16, 4\|k_tbwd" gpurun_out/${tag}_pmc.txt
