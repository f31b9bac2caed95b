# round 3 session 17: one-pass route with completion marks on demand (no event per launch):
# the multi-rank suite (one-pass exchange on 2/4 ranks, C1, C5 full size with owner/requester
# contention, stress programs), then the 2-rank exchange line beside the packed route
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s17
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 480 --timeout-method thread -m gpu tests/test_multiproc.py > gpurun_out/s17/multiproc.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s17/multiproc.log | head; tail -2 gpurun_out/s17/multiproc.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  env -u RANK -u WORLD_SIZE -u LOCAL_RANK timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s17/exchange2_onepass_$i.json 2> gpurun_out/s17/exchange2_onepass_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s17/exchange2_onepass_$i.json')); print('onepass', d['value'], d['ms_per_step'], d.get('routes'))"
done
env -u RANK -u WORLD_SIZE -u LOCAL_RANK COMEX_AMD_ONE_PASS=0 timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s17/exchange2_packed.json 2> gpurun_out/s17/exchange2_packed.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s17/exchange2_packed.json')); print('packed', d['value'], d['ms_per_step'])"
env -u RANK -u WORLD_SIZE -u LOCAL_RANK timeout -k 10 300 python -u bench.py --gpus 2 --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s17/owner_aligned2.json 2> gpurun_out/s17/owner_aligned2.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s17/owner_aligned2.json')); print('owner-aligned 2 ranks', d['value'], d['ms_per_step'])"
