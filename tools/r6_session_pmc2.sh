# SQ counters of the scaled-panel wide kernels on the current tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/r6pmc2 -o run -- python3 bench.py --config scaled --steps 4 --warmup 1 > gpurun_out/r6pmc2.log 2>&1 || { tail -5 gpurun_out/r6pmc2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r6pmc2 > gpurun_out/r6pmc2_summary.txt 2>&1 || true
rm -rf gpurun_out/r6pmc2
grep -A9 "k_mlp_fwd_zx<1\|k_tbwd_sdf<2, true>\|k_wgrad0<PrecBF16, 4, 4>" gpurun_out/r6pmc2_summary.txt
