# round 3 session 04: re-run the two multi-rank failures of s02 after the fixes, and the IPC export probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s04
P="python -u -m pytest -v --timeout 480 --timeout-method thread -m gpu"
timeout -k 10 900 $P tests/test_multiproc.py -k "one_pass or c5_full or c1" > gpurun_out/s04/mp.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/s04/mp.log | tail -12; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/ipc_export_probe.py 16 > gpurun_out/s04/ipc_probe.jsonl 2> gpurun_out/s04/ipc_probe.err
rc2=$?; cat gpurun_out/s04/ipc_probe.jsonl; tail -3 gpurun_out/s04/ipc_probe.err
exit $rc
