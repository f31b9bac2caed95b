# round 3 session 22: random multi-rank programs with the one-pass route taken by every small
# device-source accumulate into a rank of this GPU (COMEX_AMD_ONE_PASS_MIN=1): memory-lock
# hand-offs under contention, exact; then the ordinary stress and one-pass tests again
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s22
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_multiproc.py -k "stress or one_pass or c1" > gpurun_out/s22/stress.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s22/stress.log | head; tail -1 gpurun_out/s22/stress.log; exit $rc
