# round 3 session 36: does the number of rotating buffer sets (MALL defeat; SURVEY 8(d) asks for
# >= 6 sets, >= 1.2 GiB) change the headline?  driver-shaped runs with 6 / 8 / 16 sets, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/s36
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for sets in 6 8 16; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --sets $sets > $O/bench_sets${sets}_$i.json 2> $O/bench_sets${sets}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/bench_sets${sets}_$i.json')); print('sets $sets', d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['total_us'])"
  done
done
