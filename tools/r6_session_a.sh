set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tbwd_gpu.py > gpurun_out/r6a_tbwd_tests.log 2>&1 || { tail -60 gpurun_out/r6a_tbwd_tests.log; exit 1; }
tail -3 gpurun_out/r6a_tbwd_tests.log
$T 200 python3 bench.py --steps 20 --warmup 5 --no-ensemble9 > gpurun_out/r6a_bench_short.log 2>&1 || { tail -20 gpurun_out/r6a_bench_short.log; exit 1; }
tail -1 gpurun_out/r6a_bench_short.log
$T 200 python3 bench.py --no-ensemble9 > gpurun_out/r6a_bench_long.log 2>&1 || { tail -20 gpurun_out/r6a_bench_long.log; exit 1; }
tail -1 gpurun_out/r6a_bench_long.log
export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6a_prof -o run -- python3 bench.py --steps 60 --warmup 10 --no-ensemble9 > gpurun_out/r6a_prof.log 2>&1 || { tail -5 gpurun_out/r6a_prof.log; exit 1; }
python3 tools/kernel_stats.py gpurun_out/r6a_prof > gpurun_out/r6a_kernel_stats.txt 2>&1 || true
head -12 gpurun_out/r6a_kernel_stats.txt
