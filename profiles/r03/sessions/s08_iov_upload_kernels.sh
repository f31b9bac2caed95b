# round 3 session 08: io-vector upload by the copy kernel vs the runtime copy (interleaved),
# then the kernel-level GPU suite on the current tree (column kernel re-measured)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s08
export TMPDIR=/tmp
for i in 1 2; do
  for k in 1 0; do
    COMEX_AMD_IOV_KERNEL_UPLOAD=$k timeout -k 10 200 python -u tools/scatter_bench.py --pairs 16384,65536,262144 --steps 40 > gpurun_out/s08/scatter_k${k}_$i.jsonl 2> gpurun_out/s08/scatter_k${k}_$i.err || exit 1
    python -c "
import json
for l in open('gpurun_out/s08/scatter_k${k}_$i.jsonl'):
    d = json.loads(l)
    if 'pairs' in d: print('upload=$k', d['pairs'], d['ms_per_call'], d.get('cpu_reference', {}).get('ms_per_call'))"
  done
done
P="python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $P -x tests/test_gpu_parity.py tests/test_gpu_semantics.py tests/test_abi.py tests/test_legacy_acc.py > gpurun_out/s08/kernels.log 2>&1
rc=$?; tail -5 gpurun_out/s08/kernels.log; grep -i "GB/s\|gbps" gpurun_out/s08/kernels.log | head -20; exit $rc
