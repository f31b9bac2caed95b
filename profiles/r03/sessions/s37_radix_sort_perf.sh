# round 3 session 37: io-vector accumulate rate on the radix path with the library's own sort
# (hipCUB before: 1 Mi pairs 0.87-0.91 ms, 4 Mi 3.1-3.5 ms, profiles/r02/, r03/s12)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s37
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u tools/scatter_bench.py --pairs 65536,262144,1048576,4194304 --steps 20 > gpurun_out/s37/scatter_$i.jsonl 2> gpurun_out/s37/scatter_$i.err || exit 1
  python -c "
import json
for l in open('gpurun_out/s37/scatter_$i.jsonl'):
    d = json.loads(l)
    if 'pairs' in d: print(d['pairs'], d['ms_per_call'], d.get('cpu_reference', {}).get('ms_per_call'), d.get('paths'))"
done
