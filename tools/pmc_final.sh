#!/bin/bash
# PMC passes over a short sequential-graph bench run (kernel-trace only, one counter set per
# run, each within the per-block limits): instruction mix, stalls / MFMA busy, HBM bytes.
# Usage on the GPU box: bash tools/pmc_final.sh <tag> -> gpurun_out/<tag>_pmc{1,2,3}/
tag=${1:-pmcf}
cd /tmp || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export DLAP_PIPELINE=0
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM \
  --output-format csv -d $R/gpurun_out/${tag}_pmc1 -o run -- python3 $R/bench.py --steps 21 --warmup 3 --no-ensemble9 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH \
  --output-format csv -d $R/gpurun_out/${tag}_pmc2 -o run -- python3 $R/bench.py --steps 21 --warmup 3 --no-ensemble9 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES FETCH_SIZE \
  --output-format csv -d $R/gpurun_out/${tag}_pmc3 -o run -- python3 $R/bench.py --steps 21 --warmup 3 --no-ensemble9
