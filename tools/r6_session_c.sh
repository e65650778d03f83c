# new tower backward: numerics, in-kernel timing, counters, bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6c}
$T 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tbwd_gpu.py > gpurun_out/${tag}_tbwd_tests.log 2>&1 || { tail -60 gpurun_out/${tag}_tbwd_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tbwd_tests.log
$T 120 python3 tools/tbwd_probe.py --iters 20 > gpurun_out/${tag}_probe.log 2>&1 || { tail -20 gpurun_out/${tag}_probe.log; exit 1; }
grep tbwd gpurun_out/${tag}_probe.log
$T 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/${tag}_pmc1 -- python3 tools/tbwd_probe.py --iters 5 > gpurun_out/${tag}_pmc1.log 2>&1 || { tail -5 gpurun_out/${tag}_pmc1.log; exit 1; }
$T 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --output-format csv -d gpurun_out/${tag}_pmc2 -- python3 tools/tbwd_probe.py --iters 5 > gpurun_out/${tag}_pmc2.log 2>&1 || { tail -5 gpurun_out/${tag}_pmc2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/${tag}_pmc1/* gpurun_out/${tag}_pmc2/* > gpurun_out/${tag}_pmc_summary.txt 2>&1 || true
grep -A18 "tbwd" gpurun_out/${tag}_pmc_summary.txt | grep -v "^--" | head -20
for a in "--steps 20 --warmup 5" "--steps 210 --warmup 21"; do
  $T 200 python3 bench.py $a --no-ensemble9 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  tail -1 gpurun_out/${tag}_bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_epoch_phase"], d["fused_wait_timeouts"])'
done
