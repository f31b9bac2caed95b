# A/B: direct-source and packed exchange (2 ranks, one GPU, every peer treated as another
# GPU) with sched_publish_all as built (system-release events + stream sync) and as a plain
# stream sync (ab_alt/), interleaved, the round-4 conditions (300 steps, 8 sets)
set -o pipefail
out=gpurun_out/r05ab
mkdir -p $out
export COMEX_AMD_PEER_LOADS=all
for i in 1 2; do
  for v in cur alt; do
    b=bench.py; [ $v = alt ] && b=ab_alt/bench.py
    timeout -k 10 240 python3 $b --gpus 2 --exchange --src-seg --no-extras --steps 300 --warmup 20 > $out/direct_${v}_$i.json 2> $out/direct_${v}_$i.err || exit 11
    python3 -c "import json;d=json.load(open('$out/direct_${v}_$i.json'));print('direct $v', d['value'], d['ms_per_step'])"
    timeout -k 10 240 python3 $b --gpus 2 --exchange --no-extras --steps 300 --warmup 20 > $out/packed_${v}_$i.json 2> $out/packed_${v}_$i.err || exit 12
    python3 -c "import json;d=json.load(open('$out/packed_${v}_$i.json'));print('packed $v', d['value'], d['ms_per_step'])"
  done
done
