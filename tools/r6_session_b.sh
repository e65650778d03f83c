# counter passes + in-kernel timing of the SDF tower backward alone (tools/tbwd_probe.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6b}
$T 120 python3 tools/tbwd_probe.py --iters 20 > gpurun_out/${tag}_probe.log 2>&1 || { tail -20 gpurun_out/${tag}_probe.log; exit 1; }
cat gpurun_out/${tag}_probe.log
$T 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/${tag}_pmc1 -- python3 tools/tbwd_probe.py --iters 5 > gpurun_out/${tag}_pmc1.log 2>&1 || { tail -5 gpurun_out/${tag}_pmc1.log; exit 1; }
$T 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --output-format csv -d gpurun_out/${tag}_pmc2 -- python3 tools/tbwd_probe.py --iters 5 > gpurun_out/${tag}_pmc2.log 2>&1 || { tail -5 gpurun_out/${tag}_pmc2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 > gpurun_out/${tag}_pmc_summary.txt 2>&1 || true
grep -A20 "tbwd\|bwd_sdf" gpurun_out/${tag}_pmc_summary.txt | head -60
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_invariance_gpu.py -k "adam_in_tail or tail_adam_handoff or concurrent_engines or split_epoch" > gpurun_out/${tag}_inv.log 2>&1 || { tail -60 gpurun_out/${tag}_inv.log; exit 1; }
tail -8 gpurun_out/${tag}_inv.log
