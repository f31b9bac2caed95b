# r06 g: the LDS io-vector path with the multi-workgroup list read -- tests, then the A/B
set -o pipefail
o=gpurun_out/r06g
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "one_workgroup or accv or getv or putv" > $o/iov_tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/scatter_bench.py --pairs 512,1024,2048,4096,8192,16384,32768 --steps 50 --ab --nb > $o/scatter_ab.jsonl 2> $o/scatter_ab.err || exit 12
