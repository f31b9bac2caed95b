# round 3 session 10: the completion probe (how much of the closing edge a device-written
# completion flag would save), the route-toggle test after the staging-offset fix
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s10
timeout -k 10 120 ./tools/completion_probe 20 60 > gpurun_out/s10/completion.jsonl 2> gpurun_out/s10/completion.err || exit 1
timeout -k 10 120 ./tools/completion_probe 20 60 >> gpurun_out/s10/completion.jsonl 2>> gpurun_out/s10/completion.err || exit 1
timeout -k 10 120 ./tools/completion_probe 1 200 >> gpurun_out/s10/completion.jsonl 2>> gpurun_out/s10/completion.err || exit 1
cat gpurun_out/s10/completion.jsonl
P="python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $P tests/test_multiproc.py -k "toggles or selforder or self_after or remote_two or forced" > gpurun_out/s10/mp.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/s10/mp.log | tail -12; exit $rc
