# full GPU test suite of the current tree
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r6suite}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/${tag}.log 2>&1 || { tail -60 gpurun_out/${tag}.log; exit 1; }
tail -3 gpurun_out/${tag}.log
