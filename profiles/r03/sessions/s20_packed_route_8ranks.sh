# round 3 session 20: why the packed route is slow with 8 ranks sharing one GPU and every peer
# treated as another GPU (s19: C5 M2 678 ms per step packed vs 42 ms direct-source) -- HW queue
# oversubscription (8 processes x 8 streams) or the route itself?  16384^2 GA, M2 only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s20
export TMPDIR=/tmp
run() {  # name gpus env...
  local name=$1 g=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench.py --gpus $g --steps 3 --warmup 1 --warmup-ms 0 --no-cpu --ga-dims 16384 --c5-steps 2 > gpurun_out/s20/$name.json 2> gpurun_out/s20/$name.err || return 1
  python -c "
import json; d=json.load(open('gpurun_out/s20/$name.json'))['c5']
print('$name', 'M2 packed', d['M2']['ms_per_step'], 'M2 seg', d['M2_src_in_segment']['ms_per_step'], d['exchange_check']['buffer_src']['result'], d['exchange_check']['segment_src']['result'])"
}
run p8_default 8 COMEX_AMD_PEER_LOADS=all || exit 1
run p8_one_stream 8 COMEX_AMD_PEER_LOADS=all COMEX_AMD_PULL_STREAMS=0 COMEX_AMD_STREAMS=1 || exit 1
run p8_hwq1 8 COMEX_AMD_PEER_LOADS=all GPU_MAX_HW_QUEUES=1 || exit 1
run p4_default 4 COMEX_AMD_PEER_LOADS=all || exit 1
run p2_default 2 COMEX_AMD_PEER_LOADS=all || exit 1
