# round 3 session 26: one-pass floor lowered to 64 KiB (multi-rank suite), and the hand-over
# lease A/B under contention (every rank but 0 accumulating into rank 0, 3 and 5 ranks):
# COMEX_AMD_ONE_PASS_LEASE_US 0 / 100 / 400
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s26
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_multiproc.py > gpurun_out/s26/multiproc.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s26/multiproc.log | head; tail -1 gpurun_out/s26/multiproc.log; [ $rc -eq 0 ] || exit $rc
S="65536 262144 1048576 4194304"
for n in 3 5; do
  for lease in 0 100 400; do
    COMEX_AMD_ONE_PASS_LEASE_US=$lease timeout -k 10 300 python -u tools/remote_sweep.py --ranks $n --all-to-one $S > gpurun_out/s26/a2o_${n}_lease$lease.jsonl 2> gpurun_out/s26/a2o_${n}_lease$lease.err || { tail -20 gpurun_out/s26/a2o_${n}_lease$lease.err; exit 1; }
    python -c "
import json
for l in open('gpurun_out/s26/a2o_${n}_lease$lease.jsonl'):
    d=json.loads(l); print('ranks $n lease $lease', d['size'], d['us_per_op_slowest'], d['job_GBps_alg'])"
  done
done
timeout -k 10 300 python -u tools/remote_sweep.py 8192 65536 262144 1048576 > gpurun_out/s26/sweep2_floor64k.jsonl 2> gpurun_out/s26/sweep2.err || exit 1
cat gpurun_out/s26/sweep2_floor64k.jsonl
