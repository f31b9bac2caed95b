# round 3 session 18: an owner on the caller's GPU takes the one-pass route for segment
# sources too (direct-source only to other GPUs): the whole GPU suite, then the 2-rank
# exchange with the source in the segment (one-pass now) and with the route off (direct-source)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s18
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 480 --timeout-method thread -m gpu tests/ > gpurun_out/s18/gpu_suite.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s18/gpu_suite.log | head; tail -2 gpurun_out/s18/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
env -u RANK -u WORLD_SIZE -u LOCAL_RANK timeout -k 10 300 python -u bench.py --gpus 2 --exchange --src-seg --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s18/exchange2_seg_onepass.json 2> gpurun_out/s18/exchange2_seg_onepass.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s18/exchange2_seg_onepass.json')); print('segment src, one-pass', d['value'], d['ms_per_step'], d.get('routes'))"
env -u RANK -u WORLD_SIZE -u LOCAL_RANK COMEX_AMD_ONE_PASS=0 timeout -k 10 300 python -u bench.py --gpus 2 --exchange --src-seg --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s18/exchange2_seg_direct.json 2> gpurun_out/s18/exchange2_seg_direct.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s18/exchange2_seg_direct.json')); print('segment src, direct-source', d['value'], d['ms_per_step'], d.get('routes'))"
