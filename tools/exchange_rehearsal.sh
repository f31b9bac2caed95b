# 2 ranks sharing this box's one GPU: the remote accumulate path (bench --exchange, H)
# and GA_Acc of the whole array by every rank (C5 M2).  Plumbing rehearsal only:
# both "owners" live in one HBM, so nothing here measures xGMI.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 50 --warmup 5 --exchange > gpurun_out/ex_H.json 2> gpurun_out/ex_H.err || exit 1
timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --workload C5 --exchange --steps 5 --warmup 1 > gpurun_out/ex_C5.json 2> gpurun_out/ex_C5.err
