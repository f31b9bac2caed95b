# round 3 session 24: remote accumulate by message size between two ranks of one GPU
# (tools/remote_sweep.py, perf_strided-style): the one-pass floor at its default 1 MiB, at
# 1 byte (every size one-pass), and the route off (packed everywhere)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s24
export TMPDIR=/tmp
S="8192 65536 262144 1048576 4194304 16777216"
for cfg in default min1 off; do
  case $cfg in
    default) E="";;
    min1) E="COMEX_AMD_ONE_PASS_MIN=1";;
    off) E="COMEX_AMD_ONE_PASS=0";;
  esac
  env $E timeout -k 10 300 python -u tools/remote_sweep.py $S > gpurun_out/s24/sweep_$cfg.jsonl 2> gpurun_out/s24/sweep_$cfg.err || { tail -20 gpurun_out/s24/sweep_$cfg.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/s24/sweep_$cfg.jsonl'):
    d=json.loads(l); r=d['routes']; print('$cfg', d['size'], d['latency_us_median'], d['pipelined_us_per_op'], d['pipelined_GBps_alg'], 'one_pass' if r['one_pass'] else ('packed' if r['packed'] else r))"
done
