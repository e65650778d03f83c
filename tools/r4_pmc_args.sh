#!/bin/bash
# Two PMC passes (instruction mix; waits / MFMA busy / bank conflicts) over a bench run with the
# given arguments. Usage (GPU box): bash tools/r4_pmc_args.sh <tag> <bench args...>
TAG=$1; shift
cd /tmp || exit 1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export DLAP_PIPELINE=0
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM \
  --output-format csv -d $R/gpurun_out/${TAG}_pmc1 -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/${TAG}_pmc1.log 2>&1 || exit 5
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_BRANCH \
  --output-format csv -d $R/gpurun_out/${TAG}_pmc2 -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/${TAG}_pmc2.log 2>&1 || exit 6
python3 $R/tools/pmc_summary.py $R/gpurun_out/${TAG}_pmc1 $R/gpurun_out/${TAG}_pmc2 > $R/gpurun_out/${TAG}_pmc_summary.txt 2>&1
rm -rf $R/gpurun_out/${TAG}_pmc1 $R/gpurun_out/${TAG}_pmc2
grep -A18 "== void k_mlp_fwd_zx<1, false>" $R/gpurun_out/${TAG}_pmc_summary.txt
