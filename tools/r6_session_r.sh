# counters of the Gram build (and everything else) on the short bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T="timeout -k 10"
tag=${1:-r6r}
DLAP_RNN_OVERLAP=0 DLAP_SPLIT_GRAPHS=0 DLAP_TAIL_ADAM=0 $T 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/${tag}_pmc1 -- python3 bench.py --steps 40 --warmup 3 --no-ensemble9 > gpurun_out/${tag}_pmc1.log 2>&1 || { tail -5 gpurun_out/${tag}_pmc1.log; exit 1; }
DLAP_RNN_OVERLAP=0 DLAP_SPLIT_GRAPHS=0 DLAP_TAIL_ADAM=0 $T 120 rocprofv3 --pmc FETCH_SIZE TCP_TCC_READ_REQ_sum TA_BUSY_avr --output-format csv -d gpurun_out/${tag}_pmc2 -- python3 bench.py --steps 40 --warmup 3 --no-ensemble9 > gpurun_out/${tag}_pmc2.log 2>&1 || { tail -5 gpurun_out/${tag}_pmc2.log; exit 1; }
python3 tools/pmc_summary.py $(find gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 -name "*counter_collection.csv" -printf "%h\n" | sort -u) > gpurun_out/${tag}_pmc_summary.txt 2>&1 || true
rm -rf gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2
grep -A14 "k_gram" gpurun_out/${tag}_pmc_summary.txt | head -30
