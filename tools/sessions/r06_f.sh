# r06 f: plain stores in the streaming kernels -- headline bench, row-length sweep, put/get, full GPU suite
set -o pipefail
o=gpurun_out/r06f
mkdir -p $o
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench_H_1.json 2> $o/bench_H_1.err || exit 11
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu --no-host > $o/bench_H_300.json 2> $o/bench_H_300.err || exit 12
timeout -k 10 200 python tools/shape_sweep.py --rows 32,64,128,256,512,1024,2048,4096,16384 > $o/shape_sweep.jsonl 2> $o/shape_sweep.err || exit 13
timeout -k 10 200 python bench.py --xfer put --steps 50 --warmup 5 --no-cpu --no-host > $o/put_H.json 2> $o/put_H.err || exit 14
timeout -k 10 200 python bench.py --xfer get --steps 50 --warmup 5 --no-cpu --no-host > $o/get_H.json 2> $o/get_H.err || exit 15
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $o/gpu_suite.log 2>&1 || exit 16
