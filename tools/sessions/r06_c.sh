set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "one_workgroup or accv or getv or putv" > gpurun_out/r06c/iov_tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/scatter_bench.py --pairs 2048,4096,8192,16384,32768,65536 --steps 50 --ab --nb > gpurun_out/r06c/scatter_ab.jsonl 2> gpurun_out/r06c/scatter_ab.err || exit 12
timeout -k 10 500 python -u -m pytest -x -v --timeout 220 --timeout-method thread -m gpu tests/test_multiproc.py -k "xdev" > gpurun_out/r06c/xcheck_tests.log 2>&1 || exit 13
COMEX_AMD_PEER_LOADS=all timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu > gpurun_out/r06c/n2_proxy.json 2> gpurun_out/r06c/n2_proxy.err || exit 14
