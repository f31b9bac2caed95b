# A/B of asynchronous remote accumulate jobs: 4 ranks on this box's one GPU,
# C5 M2 (every rank NGA_Acc's the whole array) on a 16384^2 GA.
set -o pipefail
mkdir -p gpurun_out
for mode in 1 0 1 0; do
  COMEX_AMD_ASYNC_ACC=$mode timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port $((29550 + RANDOM % 100)) bench.py --gpus 4 --workload C5 --exchange \
    --ga-dims 16384 --steps 10 --warmup 2 > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || exit 1
  echo "async=$mode $(tail -n 1 gpurun_out/ab_$mode.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
