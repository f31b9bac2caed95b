# round 3 session 19: the driver's N = 8 invocation rehearsed on one GPU (8 ranks sharing it):
# once as is (one-pass between ranks of one GPU) and once with every peer treated as another
# GPU (COMEX_AMD_PEER_LOADS=all: packed / direct-source routes with system-scope reads, owner
# pull streams for 7 peers) -- the full C5 extras and the exchange check at 32768^2; plus the
# ARMCI message/group tests (armci_exchange_address_grp as GA's gai_get_shmem calls it)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s19
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_multiproc.py -k armci_message > gpurun_out/s19/armcimisc.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/s19/armcimisc.log | head; tail -1 gpurun_out/s19/armcimisc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --gpus 8 --steps 5 --warmup 1 --no-cpu --verbose > gpurun_out/s19/bench8_onegpu.json 2> gpurun_out/s19/bench8_onegpu.err
rc=$?; tail -c 1500 gpurun_out/s19/bench8_onegpu.json; echo; [ $rc -eq 0 ] || { tail -30 gpurun_out/s19/bench8_onegpu.err; exit $rc; }
COMEX_AMD_PEER_LOADS=all timeout -k 10 700 python -u bench.py --gpus 8 --steps 5 --warmup 1 --no-cpu --verbose > gpurun_out/s19/bench8_onegpu_peerloads.json 2> gpurun_out/s19/bench8_onegpu_peerloads.err
rc=$?; tail -c 1500 gpurun_out/s19/bench8_onegpu_peerloads.json; echo; [ $rc -eq 0 ] || { tail -30 gpurun_out/s19/bench8_onegpu_peerloads.err; exit $rc; }
