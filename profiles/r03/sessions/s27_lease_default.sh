# round 3 session 27: the one-pass lease on by default (400 us): multi-rank suite, the 2-rank
# exchange line, and the 8-rank one-GPU bench rehearsal (every rank accumulating the whole GA:
# heavy hand-over contention) at 16384^2 against the lease off
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s27
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_multiproc.py > gpurun_out/s27/multiproc.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s27/multiproc.log | head; tail -1 gpurun_out/s27/multiproc.log; [ $rc -eq 0 ] || exit $rc
env -u RANK -u WORLD_SIZE -u LOCAL_RANK timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s27/exchange2.json 2> gpurun_out/s27/exchange2.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s27/exchange2.json')); print('exchange2 one-pass', d['value'], d['hbm_peak_frac'], d['ms_per_step'])"
for lease in 400 0; do
  COMEX_AMD_ONE_PASS_LEASE_US=$lease timeout -k 10 400 python -u bench.py --gpus 8 --steps 3 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims 16384 --c5-steps 4 > gpurun_out/s27/bench8_lease$lease.json 2> gpurun_out/s27/bench8_lease$lease.err || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/s27/bench8_lease$lease.json'))['c5']
print('8 ranks lease $lease', 'M1', d['M1']['ms_per_step'], 'M2', d['M2']['ms_per_step'], 'M2 seg', d['M2_src_in_segment']['ms_per_step'], d['exchange_check']['buffer_src']['result'], d['exchange_check']['segment_src']['result'])"
done
