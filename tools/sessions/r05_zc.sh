# round-5: small io-vectors read from pinned staging without an upload launch
set -o pipefail
out=gpurun_out/r05zc
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_multiproc.py -m gpu -q -k "accv or getv or putv or io_vector or scatter or gather or stress or random_remote or vector" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/iov.log 2>&1 || { tail -30 $out/iov.log; exit 10; }
tail -1 $out/iov.log
TAG=zc bash tools/sessions/r05_iovmid.sh
cp gpurun_out/r05iovmid/accv_zc.jsonl $out/
