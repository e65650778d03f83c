export DLAP_DIST_BACKEND=gloo DLAP_SHARE_GPU=1
bash tools/gpu_round.sh \
 "bench_n2:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 105 --warmup 12" \
 "bench_n4:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 105 --warmup 12" \
 "ens_n4:300:python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 -m deeplearninginassetpricing_paperreplication_amd.parallel.ensemble --synthetic 240 60 300 3000 46 178 --epochs_unc 32 --epochs_moment 8 --epochs 64 --ignore_epoch 4"
