# round 3 session 25: the one-pass floor under contention -- every rank but 0 accumulating into
# rank 0 at once (tools/remote_sweep.py --all-to-one), one-pass at every size (floor 1 B)
# against the default floor (1 MiB: packed below), 3 and 5 ranks on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s25
export TMPDIR=/tmp
S="8192 65536 262144 1048576 4194304"
for n in 3 5; do
  for cfg in default min1; do
    E=""; [ $cfg = min1 ] && E="COMEX_AMD_ONE_PASS_MIN=1"
    env $E timeout -k 10 300 python -u tools/remote_sweep.py --ranks $n --all-to-one $S > gpurun_out/s25/a2o_${n}_$cfg.jsonl 2> gpurun_out/s25/a2o_${n}_$cfg.err || { tail -20 gpurun_out/s25/a2o_${n}_$cfg.err; exit 1; }
    python -c "
import json
for l in open('gpurun_out/s25/a2o_${n}_$cfg.jsonl'):
    d=json.loads(l); print('ranks $n $cfg', d['size'], d['us_per_op_slowest'], d['job_GBps_alg'])"
  done
done
