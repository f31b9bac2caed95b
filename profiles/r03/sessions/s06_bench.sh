# round 3 session 06: driver-shaped headline runs, rocprofv3 stats, C5 at N=1, the 2-rank
# exchange on one GPU (one-pass route now), the small io-vector crossover
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s06
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s06/bench_$i.json 2> gpurun_out/s06/bench_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/s06/bench_$i.json')); print('H', d['value'], d['hbm_peak_frac'], d['roofline']['frac'], d['value_region']['first_call_us'], d['value_region']['total_us'], d.get('blocking_api'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s06/prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/s06/prof_bench.json 2> gpurun_out/s06/prof.err || exit 1
find gpurun_out/s06/prof -name "*stats*" | head
timeout -k 10 300 python -u bench.py --gpus 1 --workload C5 --steps 10 --warmup 2 --no-cpu > gpurun_out/s06/c5_n1.json 2> gpurun_out/s06/c5_n1.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/s06/c5_n1.json')); print('C5', d['value'], d['hbm_peak_frac'], d['roofline']['frac'])"
env -u RANK -u WORLD_SIZE -u LOCAL_RANK timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s06/exchange2_onepass.json 2> gpurun_out/s06/exchange2_onepass.err || exit 1
env -u RANK -u WORLD_SIZE -u LOCAL_RANK COMEX_AMD_ONE_PASS=0 timeout -k 10 300 python -u bench.py --gpus 2 --exchange --steps 100 --warmup 5 --no-cpu --no-extras > gpurun_out/s06/exchange2_packed.json 2> gpurun_out/s06/exchange2_packed.err || exit 1
python -c "
import json
for f in ('exchange2_onepass', 'exchange2_packed'):
    d = json.load(open('gpurun_out/s06/%s.json' % f)); print(f, d['value'], d['hbm_peak_frac'])"
timeout -k 10 300 python -u tools/scatter_bench.py --pairs 16384,65536,262144 --steps 20 > gpurun_out/s06/scatter.jsonl 2> gpurun_out/s06/scatter.err || exit 1
cat gpurun_out/s06/scatter.jsonl
