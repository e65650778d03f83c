# sweep evidence on the current tree: measured bucket costs (sweep_costs.json), the full
# 384-config baseline grid and the paper grid on one GPU (full 256/64/1024 schedule)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
tag=${1:-r6n}
$T 400 python -u tools/sweep_costs.py --grid both --out gpurun_out/${tag}_sweep_costs.json > gpurun_out/${tag}_costs.log 2>&1 || { tail -20 gpurun_out/${tag}_costs.log; exit 1; }
tail -3 gpurun_out/${tag}_costs.log
for g in baseline paper; do
  $T 400 python -u -m deeplearninginassetpricing_paperreplication_amd.parallel.sweep --synthetic 240 60 300 3000 46 178 \
     --grid $g --out gpurun_out/${tag}_sweep_$g.npz > gpurun_out/${tag}_sweep_$g.log 2>&1 || { tail -20 gpurun_out/${tag}_sweep_$g.log; exit 1; }
  tail -2 gpurun_out/${tag}_sweep_$g.log | cut -c1-600
done
