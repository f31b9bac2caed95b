# round-5: accumulate rate against block size (64 MiB .. 8 GiB) on one box, then C5 N=1
set -o pipefail
out=gpurun_out/r05size
mkdir -p $out
timeout -k 10 200 python3 tools/size_probe.py > $out/size_probe.jsonl 2> $out/size_probe.err || { tail -20 $out/size_probe.err; exit 11; }
cat $out/size_probe.jsonl
timeout -k 10 300 python3 bench.py --workload C5 --no-cpu > $out/bench_C5_n1.json 2> $out/bench_C5_n1.err || exit 12
python3 -c "import json;d=json.load(open('$out/bench_C5_n1.json'));print('C5 N=1', d['value'], d['hbm_peak_frac'], d['ms_per_step'])"
