# round 3 session 16: what the system-scope (peer-GPU) loads cost on the remote routes, on one
# GPU: the 2-rank exchange with every peer treated as another GPU (COMEX_AMD_PEER_LOADS=all:
# packed route with the owner's unpack-acc reading staging by system-scope dword loads, and the
# direct-source route reading the source that way) beside the same routes with plain loads
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s16
export TMPDIR=/tmp
run() {  # name, env..., -- bench args
  local name=$1; shift
  env -u RANK -u WORLD_SIZE -u LOCAL_RANK "$@" timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 100 --warmup 5 --no-cpu --no-extras $EXTRA > gpurun_out/s16/$name.json 2> gpurun_out/s16/$name.err || return 1
  python -c "import json; d=json.load(open('gpurun_out/s16/$name.json')); print('$name', d['value'], d['hbm_peak_frac'], d['ms_per_step'], d.get('routes'))"
}
EXTRA="" run onepass COMEX_AMD_ONE_PASS=1 || exit 1
EXTRA="" run packed_plain COMEX_AMD_ONE_PASS=0 || exit 1
EXTRA="" run packed_sys COMEX_AMD_PEER_LOADS=all || exit 1
EXTRA="--src-seg" run direct_plain COMEX_AMD_ONE_PASS=1 || exit 1
EXTRA="--src-seg" run direct_sys COMEX_AMD_PEER_LOADS=all || exit 1
