# One GPU call at round end: parity suite, smoke, evidence (tools/evidence.sh),
# and a 2-rank rehearsal of the default weak-scaling bench on this box's GPU.
set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo tests ok
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo smoke ok
bash tools/evidence.sh r01
echo evidence ok
timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/bench_H_2ranks.json 2> gpurun_out/bench_H_2ranks.err
echo rehearsal ok
