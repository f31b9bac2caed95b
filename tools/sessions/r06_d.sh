set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "one_workgroup or accv or getv or putv" > gpurun_out/r06d/iov_tests.log 2>&1 || exit 11
timeout -k 10 200 python tools/scatter_bench.py --pairs 2048,4096,8192,16384,32768 --steps 50 --ab --nb > gpurun_out/r06d/scatter_ab.jsonl 2> gpurun_out/r06d/scatter_ab.err || exit 12
timeout -k 10 200 ./tools/short_rows_probe 40 > gpurun_out/r06d/short_rows_probe.jsonl 2> gpurun_out/r06d/short_rows_probe.err || exit 13
