# round 3 session 02: kernel-level GPU suite, the new multi-rank tests, the IPC export probe, the rest
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s02
P="python -u -m pytest -v --timeout 480 --timeout-method thread -m gpu"
timeout -k 10 900 $P -x tests/test_gpu_parity.py tests/test_gpu_semantics.py tests/test_abi.py tests/test_legacy_acc.py > gpurun_out/s02/kernels.log 2>&1
rc=$?; tail -3 gpurun_out/s02/kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 $P tests/test_multiproc.py -k "c1 or c5 or self_after or forced or across_devices or one_pass" > gpurun_out/s02/new_mp.log 2>&1
rc=$?; tail -3 gpurun_out/s02/new_mp.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/ipc_export_probe.py 16 > gpurun_out/s02/ipc_probe.jsonl 2> gpurun_out/s02/ipc_probe.err
rc=$?; cat gpurun_out/s02/ipc_probe.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1500 $P tests/test_multiproc.py -k "not (c1 or c5 or self_after or forced or across_devices or one_pass)" > gpurun_out/s02/rest_mp.log 2>&1
rc=$?; tail -3 gpurun_out/s02/rest_mp.log; exit $rc
