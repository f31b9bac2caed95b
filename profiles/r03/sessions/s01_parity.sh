set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_semantics.py -m gpu > gpurun_out/g1_tests.log 2>&1
rc=$?
tail -5 gpurun_out/g1_tests.log
exit $rc
