# round 3 session 41: how long the N = 8 extras take (eight ranks on one GPU, 32768^2), against the
# extras watchdog (180 s): wall time of the whole invocation and the headline part alone
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s41
export TMPDIR=/tmp
t0=$(date +%s.%N)
timeout -k 10 600 python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-extras > gpurun_out/s41/n8_noextras.json 2> gpurun_out/s41/n8_noextras.err || exit 1
t1=$(date +%s.%N)
timeout -k 10 600 python -u bench.py --gpus 8 --steps 20 --warmup 5 > gpurun_out/s41/n8_full.json 2> gpurun_out/s41/n8_full.err || exit 1
t2=$(date +%s.%N)
python -c "
import json
a, b, c = $t0, $t1, $t2
d = json.load(open('gpurun_out/s41/n8_full.json'))
print('N=8 one GPU: without extras %.1f s, with extras %.1f s (extras %.1f s); timed_out=%s; checks %s' % (b - a, c - b, (c - b) - (b - a), 'timed_out' in d['c5'], {k: v['result'] for k, v in d['c5'].get('exchange_check', {}).items()}))"
