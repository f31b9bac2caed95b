# round 3 session 40: the driver's N > 1 invocation shape exactly (torch.distributed.run, 2
# ranks; on this one-GPU box they share the card), full extras at the configured 32768^2 GA
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s40
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/s40/bench_n2.json 2> gpurun_out/s40/bench_n2.err || { tail -20 gpurun_out/s40/bench_n2.err; exit 1; }
python -c "
import json
lines = [l for l in open('gpurun_out/s40/bench_n2.json') if l.startswith('{')]
assert len(lines) == 1, len(lines)
d = json.loads(lines[0]); c = d['c5']
print('N=2 torchrun', d['value'], d['n_gpus'], d['scaling'], 'M1', c['M1']['ms_per_step'], 'M2', c['M2']['ms_per_step'], 'M2 seg', c['M2_src_in_segment']['ms_per_step'], {k: v['result'] for k, v in c['exchange_check'].items()})"
