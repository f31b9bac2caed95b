set -o pipefail
export COMEX_AMD_STAGING_MB=8
timeout -k 10 60 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29537 bench.py --gpus 2 --workload C5 --exchange --ga-dims 4096 --steps 3 --warmup 1 --verbose > gpurun_out/m2_small.json 2> gpurun_out/m2_small.err || exit 1
unset COMEX_AMD_STAGING_MB
timeout -k 10 100 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 2 --workload C5 --exchange --ga-dims 16384 --steps 2 --warmup 1 --verbose > gpurun_out/m2_mid.json 2> gpurun_out/m2_mid.err || exit 1
timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29539 bench.py --gpus 2 --workload C5 --exchange --steps 5 --warmup 1 --verbose > gpurun_out/m2_full.json 2> gpurun_out/m2_full.err
